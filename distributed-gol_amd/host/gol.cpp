// gol.cpp -- the controller ("distributor") of the host mirror, driving libgolhip.
//
// Reference flow (gol/distributor.go:194-263) and what replaces each part here:
//   read images/WxH.pgm, CellFlipped for initially alive cells  :204-216  -> same
//   rpc.Dial(broker) + makeCall/CheckStates resume              :218,69-91 -> Engine + the
//                                                                             checkpoint file
//                                                                             'q' wrote
//   Call(): per turn Broker.Publish, O(N^2) diff -> CellFlipped :45-67     -> chunked
//                                                                             golhip_step_flips
//                                                                             (per-turn flips)
//                                                                             or golhip_step(n)
//   countAliveCells: O(N^2) scan per turn, 2 s ticker           :168-191   -> per-turn counts
//                                                                             from the stencil
//   manageKeyPresses s/q/p/k                                    :105-151   -> serviced between
//                                                                             chunks
//   FinalTurnComplete, out/WxHxT.pgm, StateChange Quitting      :235-262   -> same
//
// Deliberate deviations from reference quirks, documented in
// FinalTurnComplete/StateChange carry the real completed-turn count (the reference
// always sends 0); the 's' snapshot is named with the completed turn; a tick before the first
// completed turn reports the initial count; 'q' and 'k' end Run() (closing `events`) instead of
// leaving the turn loop running.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <thread>

#include "engine.hpp"
#include "gol.hpp"

namespace gol {

std::string to_string(State s) {
    switch (s) {
        case State::Paused: return "Paused";
        case State::Executing: return "Executing";
        case State::Quitting: return "Quitting";
    }
    return "Incorrect State";
}

std::string Event::String() const {
    char buf[128];
    switch (kind) {
        case EventKind::AliveCellsCount:
            std::snprintf(buf, sizeof buf, "Alive Cells %lld", (long long)CellsCount);
            return buf;
        case EventKind::ImageOutputComplete: return "File " + Filename + " output complete";
        case EventKind::StateChange: return to_string(NewState);
        default: return "";
    }
}

Event Event::alive_cells_count(int64_t t, int64_t n) {
    Event e;
    e.kind = EventKind::AliveCellsCount;
    e.CompletedTurns = t;
    e.CellsCount = n;
    return e;
}
Event Event::image_output_complete(int64_t t, std::string f) {
    Event e;
    e.kind = EventKind::ImageOutputComplete;
    e.CompletedTurns = t;
    e.Filename = std::move(f);
    return e;
}
Event Event::state_change(int64_t t, State s) {
    Event e;
    e.kind = EventKind::StateChange;
    e.CompletedTurns = t;
    e.NewState = s;
    return e;
}
Event Event::cell_flipped(int64_t t, Cell c) {
    Event e;
    e.kind = EventKind::CellFlipped;
    e.CompletedTurns = t;
    e.cell = c;
    return e;
}
Event Event::turn_complete(int64_t t) {
    Event e;
    e.kind = EventKind::TurnComplete;
    e.CompletedTurns = t;
    return e;
}
Event Event::final_turn_complete(int64_t t, std::vector<Cell> alive) {
    Event e;
    e.kind = EventKind::FinalTurnComplete;
    e.CompletedTurns = t;
    e.Alive = std::make_shared<std::vector<Cell>>(std::move(alive));
    return e;
}

namespace {

std::vector<Cell> to_cells(const std::vector<int32_t> &xy) {
    std::vector<Cell> out(xy.size() / 2);
    for (size_t i = 0; i < out.size(); ++i) out[i] = {xy[2 * i], xy[2 * i + 1]};
    return out;
}

struct Ticker {  // gol/distributor.go:168-191 with the 2 s time.Ticker of :228
    std::mutex mu;
    int64_t turn = 0;
    int64_t count = 0;
    std::atomic<bool> stop{false};
    std::thread th;

    ~Ticker() { halt(); }  // an exception unwinding Run must not destroy a joinable thread

    void start(Channel<Event> *events, int period_ms) {
        th = std::thread([this, events, period_ms] {
            auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(period_ms);
            while (!stop.load()) {
                std::this_thread::sleep_for(std::chrono::milliseconds(5));
                if (std::chrono::steady_clock::now() < next) continue;
                next += std::chrono::milliseconds(period_ms);
                int64_t t, c;
                {
                    std::lock_guard<std::mutex> lk(mu);
                    t = turn;
                    c = count;
                }
                try {
                    events->send(Event::alive_cells_count(t, c));
                } catch (...) {
                    return;  // events closed
                }
            }
        });
    }
    void update(int64_t t, int64_t c) {
        std::lock_guard<std::mutex> lk(mu);
        turn = t;
        count = c;
    }
    void halt() {
        stop = true;
        if (th.joinable()) th.join();
    }
};

std::string board_name(const Params &p) {
    return std::to_string(p.ImageWidth) + "x" + std::to_string(p.ImageHeight);
}

void snapshot(Engine &eng, const Params &p, const RunOptions &o, const std::string &name) {
    Image img{p.ImageWidth, p.ImageHeight, eng.store()};
    write_pgm(o.out_dir + "/" + name + ".pgm", img);
}

bool file_exists(const std::string &path) {
    if (FILE *f = std::fopen(path.c_str(), "rb")) {
        std::fclose(f);
        return true;
    }
    return false;
}

void run_impl(const Params &p, Channel<Event> *events, Channel<char> *keyPresses,
              const RunOptions &o);

}  // namespace

std::string checkpoint_file(const RunOptions &o) {
    return o.checkpoint_path.empty() ? o.out_dir + "/broker_state.ckpt" : o.checkpoint_path;
}

void reset_saved_state(const RunOptions &o) { std::remove(checkpoint_file(o).c_str()); }

void Run(Params p, Channel<Event> *events, Channel<char> *keyPresses, const RunOptions &o) {
    // A failure (EngineError, I/O) ends the run the way the reference's controller ends: the
    // events channel is closed so consumers see the end, then the error propagates.
    try {
        run_impl(p, events, keyPresses, o);
    } catch (...) {
        events->close();
        throw;
    }
}

namespace {

void run_impl(const Params &p, Channel<Event> *events, Channel<char> *keyPresses,
              const RunOptions &o) {
    const std::string name = board_name(p);
    Image img = read_pgm(o.image_dir + "/" + name + ".pgm");
    if (img.width != p.ImageWidth) throw std::runtime_error("Incorrect width");
    if (img.height != p.ImageHeight) throw std::runtime_error("Incorrect height");

    int64_t turn = 0;
    const std::vector<Cell> initial = alive_cells_of(img);
    if (o.flip_events)  // gol/distributor.go:212-214
        for (const Cell &c : initial) events->send(Event::cell_flipped(0, c));

    // makeCall (gol/distributor.go:69-91): with Turns > 0, CheckStates consumes the broker's
    // paused state -- here the checkpoint file -- and resumes from it when the size matches
    // (broker/broker.go:124-141 clears `paused` either way).
    auto eng = std::make_unique<Engine>(p.ImageWidth, p.ImageHeight, o.ngpus, o.k);
    bool resumed = false;
    const std::string ckpt = checkpoint_file(o);
    if (p.Turns > 0 && file_exists(ckpt)) {
        int64_t cw = 0, ch = 0, ct = 0;
        if (golhip_checkpoint_info(ckpt.c_str(), &cw, &ch, &ct) == GOLHIP_OK && cw == p.ImageWidth &&
            ch == p.ImageHeight) {
            eng->checkpoint_load(ckpt);
            turn = ct;
            resumed = true;
        }
        std::remove(ckpt.c_str());
    }
    if (!resumed) {
        for (auto &px : img.pixels) px = px ? 255 : 0;
        eng->load(img.pixels);
    }
    eng->set_turn(turn);

    Ticker ticker;
    ticker.update(turn, turn == 0 ? (int64_t)initial.size() : (int64_t)eng->alive_count());
    ticker.start(events, o.ticker_ms);

    bool quit = false;
    // Keys (gol/distributor.go:115-148), serviced between step chunks.
    auto handle_key = [&](char key, bool &paused) {
        switch (key) {
            case 's': {
                const std::string f = name + "x" + std::to_string(turn);
                snapshot(*eng, p, o, f);
                events->send(Event::image_output_complete(turn, f));
                break;
            }
            case 'q': {
                // Pause{P: true, Turn, Dimension} parks the state in the broker (:139-147): the
                // checkpoint file outlives this process; a later Run resumes from it
                eng->checkpoint_save(ckpt);
                events->send(Event::state_change(turn, State::Quitting));
                quit = true;
                break;
            }
            case 'k': {
                const std::string f = name + "x" + std::to_string(turn);
                snapshot(*eng, p, o, f);
                events->send(Event::image_output_complete(turn, f));
                events->send(Event::state_change(turn, State::Quitting));
                eng.reset();  // Broker.Quit -> GolOP.Quit: the workers go away
                reset_saved_state(o);
                quit = true;
                break;
            }
            case 'p':
                paused = !paused;
                events->send(Event::state_change(turn, paused ? State::Paused : State::Executing));
                break;
            default: break;
        }
    };

    // Per-turn CellFlipped: chunks of turns through golhip_step_flips (each turn's flips kept in
    // a device ring, one extraction per chunk); chunk sizes grow while a chunk takes less than
    // chunk_seconds, so keys still wait at most about that long.
    const int64_t ring_cap = o.flip_events ? eng->flips_ring_capacity() : 1;
    std::vector<int32_t> fxy;
    std::vector<uint64_t> fper, falive;
    int64_t chunk = 1;
    bool paused = false;
    while (!quit && turn < p.Turns) {
        if (keyPresses) {
            while (!quit) {
                std::optional<char> key = paused ? keyPresses->recv() : keyPresses->try_recv();
                if (!key) break;
                handle_key(*key, paused);
                if (!paused) break;
            }
        }
        if (quit) break;
        const auto t0 = std::chrono::steady_clock::now();
        if (o.flip_events) {
            // per turn: CellFlipped{turn} for each flipped cell, then TurnComplete{turn+1}
            const int64_t n = std::min<int64_t>({chunk, p.Turns - turn, ring_cap});
            eng->step_flips(n, fxy, fper, falive);
            size_t at = 0;
            for (int64_t i = 0; i < n; ++i) {
                for (uint64_t c = 0; c < fper[(size_t)i]; ++c, ++at)
                    events->send(Event::cell_flipped(turn, Cell{fxy[2 * at], fxy[2 * at + 1]}));
                ++turn;
                ticker.update(turn, (int64_t)falive[(size_t)i]);
                events->send(Event::turn_complete(turn));
            }
        } else {
            const int64_t n = std::min<int64_t>(chunk, p.Turns - turn);
            const std::vector<uint64_t> c = eng->step(n, true);
            for (int64_t i = 0; i < n; ++i) {
                ticker.update(turn + i + 1, (int64_t)c[(size_t)i]);
                events->send(Event::turn_complete(turn + i + 1));
            }
            turn += n;
        }
        // chunk sized on device time + event delivery, so keys wait at most ~chunk_seconds
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt < o.chunk_seconds && chunk < (1 << 20)) chunk *= 2;
        if (dt > 4 * o.chunk_seconds && chunk > 1) chunk /= 2;
    }

    if (quit) {  // 'q' / 'k': FinalTurnComplete with no cells (gol/distributor.go:128,147)
        ticker.halt();
        events->send(Event::final_turn_complete(turn, {}));
        events->close();
        return;
    }

    std::vector<Cell> alive = to_cells(eng->alive_cells());  // gol/distributor.go:235
    ticker.halt();
    events->send(Event::final_turn_complete(turn, std::move(alive)));
    snapshot(*eng, p, o, name + "x" + std::to_string(p.Turns));  // out/WxHxT.pgm (:246-253)
    events->send(Event::state_change(turn, State::Quitting));   // :259
    events->close();                                             // :262
}

}  // namespace

int Publish(const Request &req, Response *res, int ngpus) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::unique_ptr<Engine>> cache;
    const int n = req.ImageSize;
    if (n <= 0 || (int)req.World.size() != n) return GOLHIP_ERR_ARG;
    std::vector<uint8_t> cells((size_t)n * n);
    for (int y = 0; y < n; ++y) {
        if ((int)req.World[y].size() != n) return GOLHIP_ERR_ARG;
        std::copy(req.World[y].begin(), req.World[y].end(), cells.begin() + (long)y * n);
    }
    std::lock_guard<std::mutex> lk(mu);
    auto &eng = cache[{n, ngpus}];
    if (!eng) eng = std::make_unique<Engine>(n, n, ngpus, 1);
    eng->load(cells);
    eng->step(1, false);
    const std::vector<uint8_t> out = eng->store();
    res->InitialWorld = req.World;  // broker/broker.go:158
    res->World.assign(n, std::vector<uint8_t>(n));
    for (int y = 0; y < n; ++y)
        std::copy(out.begin() + (long)y * n, out.begin() + (long)(y + 1) * n, res->World[y].begin());
    res->Turn = 1;
    return GOLHIP_OK;
}

}  // namespace gol
