// channel.hpp -- a Go-style channel for the C++ host mirror of gol.Run.
//
// The reference's controller (gol/gol.go, gol/distributor.go) is written against Go channels:
// `events chan<- Event` (unbuffered in tests, gol_test.go:33; buffered 1000 in main.go:210) and
// `keyPresses <-chan rune`.  This is the minimal equivalent: capacity 0 = rendezvous (a send
// blocks until a receiver takes the value), close() wakes every waiter, recv() on a closed and
// drained channel returns std::nullopt (Go's `v, ok := <-ch` with ok == false).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <vector>

namespace gol {

template <class T>
class Channel {
public:
    explicit Channel(std::size_t capacity = 0) : cap_(capacity) {}
    Channel(const Channel &) = delete;
    Channel &operator=(const Channel &) = delete;

    // Blocks while full (or, unbuffered, until a receiver took the value). Throws if closed.
    void send(T v) {
        std::unique_lock<std::mutex> lk(m_);
        not_full_.wait(lk, [&] { return closed_ || q_.size() < std::max<std::size_t>(cap_, 1); });
        if (closed_) throw std::runtime_error("send on closed channel");
        q_.push_back(std::move(v));
        const unsigned long long ticket = ++pushed_;
        not_empty_.notify_one();
        if (cap_ == 0) {  // rendezvous: wait until this value has been received
            taken_.wait(lk, [&] { return popped_ >= ticket || closed_; });
        }
    }

    // Sends every element of vs in order, as one send() each would, but taking the lock once per
    // run of elements that fit the buffer (a million TurnComplete events per configs[4] run: one
    // lock / wake-up per element is most of their delivery cost).  Unbuffered: one rendezvous
    // per element.  Throws if closed (elements before the close were delivered).
    void send_all(std::vector<T> &&vs) {
        if (cap_ == 0) {
            for (auto &v : vs) send(std::move(v));
            return;
        }
        std::size_t i = 0;
        std::unique_lock<std::mutex> lk(m_);
        while (i < vs.size()) {
            // a full buffer: wait until it has drained to half (pop_locked wakes this sender there),
            // then refill it in one go -- not one wake-up per element the receiver takes
            if (q_.size() >= cap_) not_full_.wait(lk, [&] { return closed_ || q_.size() <= cap_ / 2; });
            if (closed_) throw std::runtime_error("send on closed channel");
            while (i < vs.size() && q_.size() < cap_) {
                q_.push_back(std::move(vs[i++]));
                ++pushed_;
            }
            not_empty_.notify_all();
        }
    }

    std::optional<T> recv() {
        std::unique_lock<std::mutex> lk(m_);
        not_empty_.wait(lk, [&] { return closed_ || !q_.empty(); });
        return pop_locked();
    }

    // Non-blocking receive (Go's select with a default case).
    std::optional<T> try_recv() {
        std::lock_guard<std::mutex> lk(m_);
        if (q_.empty()) return std::nullopt;
        return pop_locked();
    }

    template <class Rep, class Per>
    std::optional<T> recv_for(std::chrono::duration<Rep, Per> d) {
        std::unique_lock<std::mutex> lk(m_);
        if (!not_empty_.wait_for(lk, d, [&] { return closed_ || !q_.empty(); })) return std::nullopt;
        return pop_locked();
    }

    void close() {
        std::lock_guard<std::mutex> lk(m_);
        closed_ = true;
        not_empty_.notify_all();
        not_full_.notify_all();
        taken_.notify_all();
    }

    bool closed() const {
        std::lock_guard<std::mutex> lk(m_);
        return closed_;
    }

private:
    std::optional<T> pop_locked() {
        if (q_.empty()) return std::nullopt;  // closed and drained
        T v = std::move(q_.front());
        q_.pop_front();
        ++popped_;
        // wake senders only where one can be waiting for this size: a full buffer just got room
        // (send), or it drained to half (send_all); a notify per element made the two threads
        // trade a futex wake-up for every event they passed
        const std::size_t c1 = std::max<std::size_t>(cap_, 1);
        if (q_.size() + 1 == c1 || q_.size() == c1 / 2) not_full_.notify_all();
        if (cap_ == 0) taken_.notify_all();
        return v;
    }

    std::size_t cap_;
    mutable std::mutex m_;
    std::condition_variable not_empty_, not_full_, taken_;
    std::deque<T> q_;
    bool closed_ = false;
    unsigned long long pushed_ = 0, popped_ = 0;
};

}  // namespace gol
