// test_gol_host.cpp -- the reference's integration tests, restated against the C++ host mirror
// of gol.Run (distributed-gol_amd/host) running on libgolhip.  Run from a directory holding
// images/ and check/ (tests/golden/reference); argv[1] selects the test, argv[2] = out dir.
//
//   TestGol    gol_test.go:15-47    FinalTurnComplete.Alive == alive cells of check image
//   TestPgm    pgm_test.go:10-42    out/WxHxT.pgm == check image
//   TestAlive  count_test.go:17-69  AliveCellsCount ticks match check/alive/512x512.csv
//   TestSdl    sdl_test.go:93-128   CellFlipped/TurnComplete replay a board whose count matches
//                                   the CSV every turn
//   TestKeys   s/p/q/k semantics (gol/distributor.go:105-151) incl. q -> resume (CheckStates)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <thread>

#include "../../distributed-gol_amd/host/gol.hpp"

using namespace gol;

static int g_fail = 0;
#define EXPECT(cond, ...)                                                   \
    do {                                                                    \
        if (!(cond)) {                                                      \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);       \
            std::fprintf(stderr, __VA_ARGS__);                              \
            std::fprintf(stderr, "\n");                                     \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

static std::string g_out = "out";

static std::vector<Cell> read_alive_cells(const std::string &path, int w, int h) {
    Image img = read_pgm(path);
    std::vector<Cell> cells;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            if (img.pixels[(size_t)y * w + x] != 0) cells.push_back({x, y});  // gol_test.go:119
    return cells;
}

static std::map<int, int> read_alive_counts(int w, int h) {  // count_test.go:78-89
    std::ifstream f("check/alive/" + std::to_string(w) + "x" + std::to_string(h) + ".csv");
    std::map<int, int> m;
    std::string line;
    std::getline(f, line);
    while (std::getline(f, line)) {
        int t, c;
        if (std::sscanf(line.c_str(), "%d,%d", &t, &c) == 2) m[t] = c;
    }
    return m;
}

static bool same_board(std::vector<Cell> a, std::vector<Cell> b) {  // multiset, gol_test.go:58-86
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    return a == b;
}

static RunOptions opts() {
    RunOptions o;
    o.out_dir = g_out;
    return o;
}

static void test_gol(bool pgm) {
    for (int n : {16, 64, 512}) {
        for (int turns : {0, 1, 100}) {
            const std::string exp_path = "check/images/" + std::to_string(n) + "x" +
                                         std::to_string(n) + "x" + std::to_string(turns) + ".pgm";
            const auto expected = read_alive_cells(exp_path, n, n);
            std::vector<int> threads_list;
            for (int t = 1; t <= 16; ++t)
                if (n < 512 || t == 1 || t == 8 || t == 16) threads_list.push_back(t);
            for (int threads : threads_list) {
                Params p{turns, threads, n, n};
                Channel<Event> events(1024);
                std::thread th([&] { Run(p, &events, nullptr, opts()); });
                std::vector<Cell> cells;
                bool final_seen = false;
                while (auto e = events.recv()) {
                    if (e->kind == EventKind::FinalTurnComplete) {
                        cells = *e->Alive;
                        final_seen = true;
                        EXPECT(e->CompletedTurns == turns, "final turn %lld != %d",
                               (long long)e->CompletedTurns, turns);
                    }
                }
                th.join();
                EXPECT(final_seen, "%dx%dx%d-%d: no FinalTurnComplete", n, n, turns, threads);
                if (!pgm) {
                    EXPECT(same_board(cells, expected), "%dx%dx%d-%d: board mismatch", n, n, turns, threads);
                } else {
                    const std::string out = g_out + "/" + std::to_string(n) + "x" + std::to_string(n) +
                                            "x" + std::to_string(turns) + ".pgm";
                    EXPECT(same_board(read_alive_cells(out, n, n), expected), "%s mismatch", out.c_str());
                    // byte-identical file, header included (gol/io.go:52-59)
                    std::ifstream a(out, std::ios::binary), b(exp_path, std::ios::binary);
                    std::string sa((std::istreambuf_iterator<char>(a)), {}), sb((std::istreambuf_iterator<char>(b)), {});
                    EXPECT(sa == sb, "%s not byte-identical to %s", out.c_str(), exp_path.c_str());
                }
            }
        }
    }
}

static void test_alive() {
    Params p{100000000, 8, 512, 512};
    auto alive = read_alive_counts(512, 512);
    Channel<Event> events(0);  // unbuffered, as count_test.go:154
    Channel<char> keys(2);
    RunOptions o = opts();
    o.flip_events = false;
    std::thread th([&] { Run(p, &events, &keys, o); });
    const auto t0 = std::chrono::steady_clock::now();
    int i = 0;
    bool quit_sent = false;
    while (auto e = events.recv()) {
        if (e->kind == EventKind::AliveCellsCount && !quit_sent) {
            if (i == 0) {
                const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                EXPECT(dt < 5.0, "no AliveCellsCount within 5 s (%.2f s)", dt);
            }
            int expected;
            if (e->CompletedTurns <= 10000)
                expected = e->CompletedTurns == 0 ? 6511 : alive[e->CompletedTurns];
            else
                expected = e->CompletedTurns % 2 == 0 ? 5565 : 5567;
            EXPECT(expected == e->CellsCount, "At turn %lld expected %d alive cells, got %lld",
                   (long long)e->CompletedTurns, expected, (long long)e->CellsCount);
            std::printf("Completed Turns %-8lld%s\n", (long long)e->CompletedTurns, e->String().c_str());
            if (++i >= 5) {
                keys.send('q');
                quit_sent = true;
            }
        }
    }
    th.join();
    EXPECT(i >= 5, "not enough AliveCellsCount events received");
    reset_saved_state(opts());
}

static void test_sdl() {
    Params p{100, 8, 512, 512};
    auto alive = read_alive_counts(512, 512);
    Channel<Event> events(0);
    std::thread th([&] { Run(p, &events, nullptr, opts()); });
    std::vector<uint8_t> board(512 * 512, 0);
    int turn_num = 0;
    bool final = false;
    while (auto e = events.recv()) {
        switch (e->kind) {
            case EventKind::CellFlipped: {
                uint8_t &b = board[(size_t)e->cell.Y * 512 + e->cell.X];
                b = (uint8_t)~b;  // sdl_test.go:58
                break;
            }
            case EventKind::TurnComplete: {
                ++turn_num;
                const int count = (int)std::count(board.begin(), board.end(), (uint8_t)255);
                EXPECT(alive[turn_num] == count, "turn %d: displayed %d alive, should be %d",
                       turn_num, count, alive[turn_num]);
                EXPECT(e->CompletedTurns == turn_num, "TurnComplete %lld != %d",
                       (long long)e->CompletedTurns, turn_num);
                break;
            }
            case EventKind::FinalTurnComplete: final = true; break;
            default: break;
        }
    }
    th.join();
    EXPECT(final, "Simulation finished without sending a FinalTurnComplete event.");
    EXPECT(turn_num == 100, "saw %d TurnComplete events", turn_num);
}

static void test_keys() {
    // p: pause / resume events; s: snapshot file; q: park, then a new Run resumes (CheckStates)
    Params p{1000000, 8, 512, 512};
    Channel<Event> events(4096);
    Channel<char> keys(8);
    RunOptions o = opts();
    o.flip_events = false;
    std::thread th([&] { Run(p, &events, &keys, o); });
    std::vector<Event> seen;
    int snap_turn = -1, quit_turn = -1;
    bool sent = false;
    while (auto e = events.recv()) {
        if (!sent && e->kind == EventKind::TurnComplete && e->CompletedTurns >= 50) {
            keys.send('p');
            keys.send('s');
            keys.send('p');
            keys.send('q');
            sent = true;
        }
        if (e->kind == EventKind::StateChange || e->kind == EventKind::ImageOutputComplete) {
            seen.push_back(*e);
            std::printf("Completed Turns %-8lld%s\n", (long long)e->CompletedTurns, e->String().c_str());
        }
        if (e->kind == EventKind::ImageOutputComplete) snap_turn = (int)e->CompletedTurns;
        if (e->kind == EventKind::StateChange && e->NewState == State::Quitting) quit_turn = (int)e->CompletedTurns;
    }
    th.join();
    EXPECT(seen.size() == 4, "expected Paused, snapshot, Executing, Quitting; got %zu", seen.size());
    if (seen.size() == 4) {
        EXPECT(seen[0].NewState == State::Paused, "first state change not Paused");
        EXPECT(seen[1].kind == EventKind::ImageOutputComplete, "snapshot event missing");
        EXPECT(seen[2].NewState == State::Executing, "no Executing after second p");
        EXPECT(seen[3].NewState == State::Quitting, "no Quitting after q");
        EXPECT(seen[0].CompletedTurns == seen[1].CompletedTurns, "snapshot taken while paused");
    }
    // the snapshot is the board at snap_turn: checked against the CSV count
    auto alive = read_alive_counts(512, 512);
    if (snap_turn > 0) {
        const std::string f = g_out + "/512x512x" + std::to_string(snap_turn) + ".pgm";
        const int c = (int)read_alive_cells(f, 512, 512).size();
        const int exp = snap_turn <= 10000 ? alive[snap_turn] : (snap_turn % 2 ? 5567 : 5565);
        EXPECT(c == exp, "snapshot %s has %d alive, expected %d", f.c_str(), c, exp);
    }
    std::printf("snapshot turn %d, quit turn %d\n", snap_turn, quit_turn);
    // resume: same size, the parked board continues from quit_turn (gol/distributor.go:79-84)
    Params p2{quit_turn + 10, 8, 512, 512};
    Channel<Event> ev2(4096);
    std::thread th2([&] { Run(p2, &ev2, nullptr, o); });
    int first_turn = -1, final_turn = -1;
    size_t final_cells = 0;
    while (auto e = ev2.recv()) {
        if (e->kind == EventKind::TurnComplete && first_turn < 0) first_turn = (int)e->CompletedTurns;
        if (e->kind == EventKind::FinalTurnComplete) {
            final_turn = (int)e->CompletedTurns;
            final_cells = e->Alive->size();
        }
    }
    th2.join();
    EXPECT(first_turn == quit_turn + 1, "resumed at %d, expected %d", first_turn, quit_turn + 1);
    EXPECT(final_turn == quit_turn + 10, "final turn %d", final_turn);
    const int t = quit_turn + 10;
    const int exp = t <= 10000 ? alive[t] : (t % 2 ? 5567 : 5565);
    EXPECT((int)final_cells == exp, "resumed board has %zu alive at turn %d, expected %d",
           final_cells, t, exp);
    // k: snapshot + quit, nothing parked afterwards
    Params p3{1000000, 8, 64, 64};
    Channel<Event> ev3(4096);
    Channel<char> k3(2);
    std::thread th3([&] { Run(p3, &ev3, &k3, o); });
    bool ksent = false, quitting = false;
    while (auto e = ev3.recv()) {
        if (!ksent && e->kind == EventKind::TurnComplete) {
            k3.send('k');
            ksent = true;
        }
        if (e->kind == EventKind::StateChange && e->NewState == State::Quitting) quitting = true;
    }
    th3.join();
    EXPECT(quitting, "k did not quit");
}

static void test_publish() {
    // Broker.Publish contract (broker/broker.go:157-180): World -> next generation
    Image img = read_pgm("images/64x64.pgm");
    Request req;
    req.ImageSize = 64;
    req.World.assign(64, std::vector<uint8_t>(64));
    for (int y = 0; y < 64; ++y)
        for (int x = 0; x < 64; ++x) req.World[y][x] = img.pixels[(size_t)y * 64 + x];
    Response res;
    EXPECT(Publish(req, &res) == 0, "Publish failed");
    Image exp = read_pgm("check/images/64x64x1.pgm");
    bool ok = res.InitialWorld == req.World;
    for (int y = 0; y < 64; ++y)
        for (int x = 0; x < 64; ++x) ok = ok && res.World[y][x] == exp.pixels[(size_t)y * 64 + x];
    EXPECT(ok, "Publish result differs from check/images/64x64x1.pgm");
}

int main(int argc, char **argv) {
    const std::string which = argc > 1 ? argv[1] : "all";
    if (argc > 2) g_out = argv[2];
    const auto t0 = std::chrono::steady_clock::now();
    if (which == "TestGol" || which == "all") test_gol(false);
    if (which == "TestPgm" || which == "all") test_gol(true);
    if (which == "TestAlive" || which == "all") test_alive();
    if (which == "TestSdl" || which == "all") test_sdl();
    if (which == "TestKeys" || which == "all") test_keys();
    if (which == "TestPublish" || which == "all") test_publish();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%s: %s (%d failures, %.2f s)\n", which.c_str(), g_fail ? "FAIL" : "ok", g_fail, dt);
    return g_fail ? 1 : 0;
}
