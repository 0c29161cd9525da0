// host_bench.cpp -- configs[4]'s own metric: the host contract (gol::Run) timed as a consumer sees it.
//
// The reference's controller serves an SDL window and a key loop while it runs (gol/distributor.go:
// 105-151 keys, :168-191 the 2 s AliveCellsCount ticker; sdl/loop.go:9-54 the consumer).  This
// program is that consumer: it runs gol::Run on images/<W>x<H>.pgm with per-turn TurnComplete (and
// optionally CellFlipped) events, presses keys at scheduled times, and reports
//   * turns/s with every TurnComplete received (wall, and with the paused time taken out);
//   * tick latency: AliveCellsCount fired (Event::FiredNs) -> received here, median / p90 / max;
//   * key latency: key sent -> its StateChange / ImageOutputComplete received;
//   * every tick's count and the final count against the expected per-turn counts (the oracle's
//     golden, written by bench.py as uint32 counts of turns 0..T), TurnComplete in order, and the
//     's' snapshot file's alive cells against the count of its turn.
// One JSON line on stdout.  Usage:
//   host_bench -w W -h H -turns T -images DIR -out DIR -expected FILE [-ticker_ms 2000]
//              [-keys p@0.4,s@0.6,p@1.2] [-flips] [-depth 2] [-chunk_s 0.02]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "gol.hpp"

using namespace gol;
using Clock = std::chrono::steady_clock;

namespace {

int64_t ns_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

struct KeyAt {
    char key;
    double at_s;
};

std::vector<KeyAt> parse_keys(const std::string &spec) {
    std::vector<KeyAt> out;
    size_t i = 0;
    while (i < spec.size()) {
        size_t j = spec.find(',', i);
        if (j == std::string::npos) j = spec.size();
        const std::string tok = spec.substr(i, j - i);
        if (tok.size() >= 3 && tok[1] == '@') out.push_back({tok[0], std::atof(tok.c_str() + 2)});
        i = j + 1;
    }
    return out;
}

double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5))];
}

}  // namespace

int main(int argc, char **argv) {
    Params p{1000000, 8, 4096, 4096};
    RunOptions o;
    o.flip_events = false;
    o.k = 16;
    std::string expected_path, keyspec;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : "0"; };
        if (a == "-w") p.ImageWidth = std::atoi(next());
        else if (a == "-h") p.ImageHeight = std::atoi(next());
        else if (a == "-turns") p.Turns = std::strtoll(next(), nullptr, 10);
        else if (a == "-images") o.image_dir = next();
        else if (a == "-out") o.out_dir = next();
        else if (a == "-expected") expected_path = next();
        else if (a == "-ticker_ms") o.ticker_ms = std::atoi(next());
        else if (a == "-keys") keyspec = next();
        else if (a == "-flips") o.flip_events = true;
        else if (a == "-depth") o.pipeline_depth = std::atoi(next());
        else if (a == "-chunk_s") o.chunk_seconds = std::atof(next());
    }
    std::vector<uint32_t> expected;
    if (!expected_path.empty()) {
        std::ifstream f(expected_path, std::ios::binary);
        f.seekg(0, std::ios::end);
        expected.resize((size_t)f.tellg() / 4);
        f.seekg(0);
        f.read(reinterpret_cast<char *>(expected.data()), (std::streamsize)(expected.size() * 4));
    }
    auto exp_at = [&](int64_t t) -> int64_t { return t >= 0 && (size_t)t < expected.size() ? (int64_t)expected[(size_t)t] : -1; };
    reset_saved_state(o);  // a fresh board, not a parked one

    Channel<Event> events(1000);  // main.go:210
    Channel<char> keys(10);       // main.go:209
    const std::vector<KeyAt> plan = parse_keys(keyspec);
    std::vector<int64_t> key_sent_ns(plan.size(), 0);
    const int64_t t0 = ns_now();
    std::thread run([&] {
        try {
            Run(p, &events, &keys, o);
        } catch (const std::exception &e) {
            std::fprintf(stderr, "host_bench: Run failed: %s\n", e.what());
            std::_Exit(2);
        }
    });
    std::thread presser([&] {  // the SDL key loop's role (sdl/loop.go:17-27)
        for (size_t i = 0; i < plan.size(); ++i) {
            std::this_thread::sleep_until(Clock::time_point(std::chrono::nanoseconds(t0)) +
                                          std::chrono::duration_cast<Clock::duration>(
                                              std::chrono::duration<double>(plan[i].at_s)));
            key_sent_ns[i] = ns_now();
            try {
                keys.send(plan[i].key);
            } catch (...) {
                return;
            }
        }
    });

    int64_t turn_completes = 0, last_tc = 0, flips = 0, final_turn = -1, final_alive = -1;
    bool in_order = true;
    std::vector<double> tick_ms;
    int64_t ticks = 0, tick_bad = 0;
    std::string tick_first_bad;
    struct KeyEv {
        std::string what;
        int64_t turn;
        int64_t recv_ns;
    };
    std::vector<KeyEv> key_events;
    int64_t paused_ns = 0, paused_at = -1, first_tc_ns = 0, last_tc_ns = 0;
    std::string snapshot;
    int64_t snapshot_turn = -1;
    while (auto e = events.recv()) {
        if (e->kind == EventKind::CellFlipped) {  // the bulk of a flips run: no clock read
            ++flips;
            continue;
        }
        const int64_t now = ns_now();
        switch (e->kind) {
            case EventKind::TurnComplete:
                ++turn_completes;
                if (e->CompletedTurns != last_tc + 1) in_order = false;
                last_tc = e->CompletedTurns;
                if (!first_tc_ns) first_tc_ns = now;
                last_tc_ns = now;
                break;
            case EventKind::CellFlipped: break;
            case EventKind::AliveCellsCount: {
                ++ticks;
                tick_ms.push_back((double)(now - e->FiredNs) * 1e-6);
                const int64_t want = exp_at(e->CompletedTurns);
                if (want != e->CellsCount) {
                    if (!tick_bad)
                        tick_first_bad = "turn " + std::to_string(e->CompletedTurns) + ": " +
                                         std::to_string(e->CellsCount) + " != " + std::to_string(want);
                    ++tick_bad;
                }
                break;
            }
            case EventKind::StateChange:
                key_events.push_back({to_string(e->NewState), e->CompletedTurns, now});
                if (e->NewState == State::Paused) paused_at = now;
                if (e->NewState == State::Executing && paused_at >= 0) {
                    paused_ns += now - paused_at;
                    paused_at = -1;
                }
                break;
            case EventKind::ImageOutputComplete:
                key_events.push_back({"ImageOutputComplete", e->CompletedTurns, now});
                snapshot = e->Filename;
                snapshot_turn = e->CompletedTurns;
                break;
            case EventKind::FinalTurnComplete:
                final_turn = e->CompletedTurns;
                final_alive = e->Alive ? (int64_t)e->Alive->size() : -1;
                break;
        }
    }
    const int64_t t_end = ns_now();
    run.join();
    presser.join();

    // match each scheduled key to the first event of its kind received after it was sent
    std::string keys_json = "[";
    std::vector<bool> used(key_events.size(), false);
    for (size_t i = 0; i < plan.size(); ++i) {
        const char *want = plan[i].key == 's' ? "ImageOutputComplete" : nullptr;
        double lat = -1.0;
        std::string ev;
        int64_t turn = -1;
        for (size_t j = 0; j < key_events.size(); ++j) {
            if (used[j] || key_events[j].recv_ns < key_sent_ns[i]) continue;
            const bool ok = want ? key_events[j].what == want
                                 : (key_events[j].what == "Paused" || key_events[j].what == "Executing" ||
                                    key_events[j].what == "Quitting");
            if (!ok) continue;
            used[j] = true;
            lat = (double)(key_events[j].recv_ns - key_sent_ns[i]) * 1e-6;
            ev = key_events[j].what;
            turn = key_events[j].turn;
            break;
        }
        char buf[256];
        std::snprintf(buf, sizeof buf, "%s{\"key\": \"%c\", \"at_s\": %.3f, \"event\": \"%s\", \"turn\": %lld, \"latency_ms\": %.3f}",
                      i ? ", " : "", plan[i].key, plan[i].at_s, ev.c_str(), (long long)turn, lat);
        keys_json += buf;
    }
    keys_json += "]";

    // the 's' snapshot file: its alive cells against the count of its turn
    int64_t snap_alive = -1;
    if (!snapshot.empty()) {
        Image img = read_pgm(o.out_dir + "/" + snapshot + ".pgm");
        snap_alive = (int64_t)alive_cells_of(img).size();
    }
    const double wall = (double)(t_end - t0) * 1e-9;
    const double active = wall - (double)paused_ns * 1e-9;
    const double tc_span = (double)(last_tc_ns - first_tc_ns) * 1e-9;
    // streaming rate: first to last TurnComplete received, the paused time taken out (wall_s also
    // holds the start-up: PGM read, engine create, board load, the first chunks' graph captures)
    const double streaming = tc_span - (double)paused_ns * 1e-9;
    std::printf(
        "{\"board\": \"%dx%d\", \"turns\": %lld, \"ticker_ms\": %d, \"pipeline_depth\": %d, \"flip_events\": %s, "
        "\"wall_s\": %.4f, \"paused_s\": %.4f, \"active_s\": %.4f, \"turns_per_s_active\": %.1f, "
        "\"us_per_turn_active\": %.4f, \"turn_complete_span_s\": %.4f, \"us_per_turn_streaming\": %.4f, "
        "\"turns_per_s_streaming\": %.1f, "
        "\"turn_complete\": {\"n\": %lld, \"in_order\": %s}, \"cell_flipped\": %lld, "
        "\"ticks\": {\"n\": %lld, \"latency_ms_median\": %.3f, \"latency_ms_p90\": %.3f, \"latency_ms_max\": %.3f, "
        "\"counts_match\": %s, \"mismatches\": %lld, \"first_mismatch\": \"%s\"}, "
        "\"keys\": %s, \"snapshot\": {\"file\": \"%s\", \"turn\": %lld, \"alive\": %lld, \"match\": %s}, "
        "\"final\": {\"turn\": %lld, \"alive\": %lld, \"match\": %s}}\n",
        p.ImageWidth, p.ImageHeight, (long long)p.Turns, o.ticker_ms, o.pipeline_depth, o.flip_events ? "true" : "false",
        wall, (double)paused_ns * 1e-9, active, (double)p.Turns / active, active / (double)p.Turns * 1e6, tc_span,
        streaming / (double)p.Turns * 1e6, (double)p.Turns / streaming,
        (long long)turn_completes, in_order && turn_completes == p.Turns ? "true" : "false", (long long)flips,
        (long long)ticks, pct(tick_ms, 0.5), pct(tick_ms, 0.9), pct(tick_ms, 1.0),
        tick_bad == 0 && !expected.empty() ? "true" : "false", (long long)tick_bad, tick_first_bad.c_str(),
        keys_json.c_str(), snapshot.c_str(), (long long)snapshot_turn, (long long)snap_alive,
        snapshot.empty() ? "null" : (snap_alive == exp_at(snapshot_turn) ? "true" : "false"),
        (long long)final_turn, (long long)final_alive, final_alive == exp_at(final_turn) ? "true" : "false");
    std::fflush(stdout);
    return 0;
}
