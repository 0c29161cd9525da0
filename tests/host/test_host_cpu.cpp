// test_host_cpu.cpp -- CPU-only unit tests of the C++ host mirror (no device calls):
// the Go-style channel (gol/gol.go wires unbuffered channels, gol/gol.go:48-54) and the PGM
// codec (gol/io.go:42-128), checked byte-exact against the reference's fixtures.
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../distributed-gol_amd/host/gol.hpp"

using namespace gol;
static int g_fail = 0;
#define EXPECT(c, msg)                                                     \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, msg); \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

static std::string slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    return std::string((std::istreambuf_iterator<char>(f)), {});
}

int main(int argc, char **argv) {
    const std::string ref = argc > 1 ? argv[1] : "tests/golden/reference";
    const std::string tmp = argc > 2 ? argv[2] : "/tmp";
    // unbuffered channel: send completes only after the receive
    {
        Channel<int> ch(0);
        bool received = false;
        std::thread t([&] {
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
            auto v = ch.recv();
            received = v && *v == 7;
        });
        ch.send(7);
        t.join();
        EXPECT(received, "rendezvous value lost");
        ch.close();
        EXPECT(!ch.recv().has_value(), "recv on closed channel must report !ok");
        bool threw = false;
        try { ch.send(1); } catch (...) { threw = true; }
        EXPECT(threw, "send on closed channel must fail");
    }
    // buffered channel keeps order and drains after close
    {
        Channel<int> ch(4);
        for (int i = 0; i < 4; ++i) ch.send(i);
        ch.close();
        for (int i = 0; i < 4; ++i) EXPECT(ch.recv().value_or(-1) == i, "fifo order");
        EXPECT(!ch.recv(), "drained");
        EXPECT(!ch.try_recv(), "try_recv on empty");
    }
    // send_all: one batch through a small buffer, received in order by a slower consumer
    // (the delivery thread's TurnComplete slices, host/gol.cpp Pipeline); unbuffered: rendezvous each
    for (size_t cap : {size_t(0), size_t(3), size_t(1000)}) {
        Channel<int> ch(cap);
        std::vector<int> got;
        std::thread t([&] {
            while (auto v = ch.recv()) got.push_back(*v);
        });
        std::vector<int> batch;
        for (int i = 0; i < 5000; ++i) batch.push_back(i);
        ch.send_all(std::move(batch));
        ch.send_all({5000, 5001});
        ch.close();
        t.join();
        bool ordered = got.size() == 5002;
        for (size_t i = 0; ordered && i < got.size(); ++i) ordered = got[i] == (int)i;
        EXPECT(ordered, "send_all lost or reordered elements");
        bool threw = false;
        try { ch.send_all({1}); } catch (...) { threw = true; }
        EXPECT(threw, "send_all on closed channel must fail");
    }
    // two senders at once -- the delivery thread's send_all batches and the ticker's single sends --
    // into a small buffer, a receiver slower than both: nothing lost, each sender's order kept, no
    // sender left waiting (a full buffer wakes its waiters at room and at half: channel.hpp)
    for (size_t cap : {size_t(1), size_t(7), size_t(64)}) {
        Channel<int> ch(cap);
        std::vector<int> got;
        std::thread rx([&] {
            int n = 0;
            while (auto v = ch.recv()) {
                got.push_back(*v);
                if (++n % 97 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
        });
        std::thread tick([&] {
            for (int i = 0; i < 300; ++i) ch.send(1000000 + i);
        });
        for (int b = 0; b < 40; ++b) {
            std::vector<int> batch;
            for (int i = 0; i < 250; ++i) batch.push_back(b * 250 + i);
            ch.send_all(std::move(batch));
        }
        tick.join();
        ch.close();
        rx.join();
        int next_batch = 0, next_tick = 1000000;
        bool ok = got.size() == 10000 + 300;
        for (int v : got) {
            if (v >= 1000000) ok = ok && v == next_tick++;
            else ok = ok && v == next_batch++;
        }
        EXPECT(ok, "two senders: lost or reordered elements");
    }
    // PGM round trip, byte-exact with the reference's files (header "P5\n<W> <H>\n255\n")
    for (const char *n : {"16x16", "64x64", "512x512"}) {
        const std::string in = ref + "/images/" + n + ".pgm";
        Image img = read_pgm(in);
        const std::string out = tmp + "/golhost_" + n + ".pgm";
        write_pgm(out, img);
        EXPECT(slurp(in) == slurp(out), "pgm round trip not byte-exact");
    }
    Image g = read_pgm(ref + "/images/16x16.pgm");
    EXPECT(alive_cells_of(g).size() == 5, "16x16 holds a 5-cell glider");
    Image b = read_pgm(ref + "/images/64x64.pgm");
    EXPECT(alive_cells_of(b).size() == 2819, "64x64 initial alive count");
    // events print like the reference (gol/event.go:71-131)
    EXPECT(Event::alive_cells_count(3, 42).String() == "Alive Cells 42", "AliveCellsCount string");
    EXPECT(Event::state_change(1, State::Paused).String() == "Paused", "StateChange string");
    EXPECT(Event::turn_complete(1).String().empty(), "TurnComplete prints nothing");
    std::printf("host cpu tests: %s\n", g_fail ? "FAIL" : "ok");
    return g_fail ? 1 : 0;
}
