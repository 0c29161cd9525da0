// engine.hpp -- RAII C++ wrapper over the libgolhip C ABI (include/golhip.h).
// Host code only: no HIP headers, exactly what a cgo/JNI/ctypes caller would see.
#pragma once

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/golhip.h"

namespace gol {

struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

class Engine {
public:
    Engine(int width, int height, int ngpus, int k) {
        const int rc = golhip_create(width, height, ngpus, k, &h_);
        if (rc != GOLHIP_OK)
            throw EngineError(rc, std::string("golhip_create: ") + golhip_strerror(rc));
        check(golhip_get_info(h_, &info_));
    }
    ~Engine() {
        if (h_) golhip_destroy(h_);
    }
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;

    const golhip_info &info() const { return info_; }

    void load(const std::vector<uint8_t> &cells) {
        check(golhip_load_bytes(h_, cells.data(), (size_t)info_.width));
    }
    std::vector<uint8_t> store() {
        std::vector<uint8_t> out((size_t)info_.width * (size_t)info_.rows);
        check(golhip_store_bytes(h_, out.data(), (size_t)info_.width));
        return out;
    }
    // Advance `turns`; returns the alive count after each turn when `counts`.
    std::vector<uint64_t> step(int64_t turns, bool counts) {
        std::vector<uint64_t> c(counts ? (size_t)turns : 0);
        check(golhip_step(h_, turns, counts ? c.data() : nullptr));
        return c;
    }
    void set_k(int k) { check(golhip_set_k(h_, k)); }
    uint64_t alive_count() {
        uint64_t v = 0;
        check(golhip_alive_count(h_, &v));
        return v;
    }
    std::vector<int32_t> alive_cells() { return cells(golhip_alive_cells); }
    std::vector<int32_t> flips() { return cells(golhip_flips); }
    // Per-turn flips of `turns` turns (<= flips_ring_capacity()): xy = every turn's cells, turn
    // by turn; per_turn[t] = cells of turn t; alive[t] = alive after turn t.
    void step_flips(int64_t turns, std::vector<int32_t> &xy, std::vector<uint64_t> &per_turn,
                    std::vector<uint64_t> &alive) {
        per_turn.resize((size_t)turns);
        alive.resize((size_t)turns);
        size_t n = 0;
        if (xy.size() < 2) xy.resize(2 << 16);
        int rc = golhip_step_flips(h_, turns, xy.data(), xy.size() / 2, &n, per_turn.data(),
                                   alive.data());
        if (rc == GOLHIP_ERR_CAP) {  // the turns ran; fetch into a larger list
            xy.resize(2 * std::max(n, xy.size()));
            rc = golhip_flips_fetch(h_, xy.data(), xy.size() / 2, &n, per_turn.data());
        }
        check(rc);
    }
    int64_t flips_ring_capacity() {
        int64_t c = 1;
        check(golhip_flips_ring_capacity(h_, &c));
        return c;
    }
    void track_flips(bool on) { check(golhip_track_flips(h_, on ? 1 : 0)); }
    void checkpoint_save(const std::string &path) { check(golhip_checkpoint_save(h_, path.c_str())); }
    void checkpoint_load(const std::string &path) { check(golhip_checkpoint_load(h_, path.c_str())); }
    int64_t turn() {
        int64_t t = 0;
        check(golhip_turn(h_, &t));
        return t;
    }
    void set_turn(int64_t t) { check(golhip_set_turn(h_, t)); }
    void sync() { check(golhip_sync(h_)); }

private:
    template <class F>
    std::vector<int32_t> cells(F fn) {
        size_t n = 0;
        int rc = fn(h_, nullptr, 0, &n);
        if (rc != GOLHIP_OK && rc != GOLHIP_ERR_CAP) check(rc);
        std::vector<int32_t> xy(2 * n);
        check(fn(h_, xy.data(), n, &n));
        xy.resize(2 * n);
        return xy;
    }
    void check(int rc) {
        if (rc != GOLHIP_OK)
            throw EngineError(rc, std::string(golhip_strerror(rc)) + ": " + golhip_last_error(h_));
    }
    golhip_t h_ = nullptr;
    golhip_info info_{};
};

}  // namespace gol
