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
//   the unbuffered channels that make the turn loop wait for   gol/gol.go:48-54 -> a delivery
//   every consumer each turn                                                   thread: chunk n's
//                                                                             events go out while
//                                                                             chunk n+1 runs
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
#include <condition_variable>
#include <exception>
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

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Ticker {  // gol/distributor.go:168-191 with the 2 s time.Ticker of :228
    std::mutex mu;
    std::condition_variable cv;
    int64_t turn = 0;
    int64_t count = 0;
    bool stop = false;
    std::thread th;

    ~Ticker() { halt(); }  // an exception unwinding Run must not destroy a joinable thread

    void start(Channel<Event> *events, int period_ms) {
        th = std::thread([this, events, period_ms] {
            auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(period_ms);
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                // sleep to the tick itself (no polling granularity in the tick latency)
                if (cv.wait_until(lk, next, [&] { return stop; })) return;
                const int64_t fired = now_ns();
                next += std::chrono::milliseconds(period_ms);
                Event e = Event::alive_cells_count(turn, count);
                e.FiredNs = fired;
                lk.unlock();
                try {
                    events->send(std::move(e));
                } catch (...) {
                    return;  // events closed
                }
                lk.lock();
            }
        });
    }
    // the latch of gol/distributor.go:180-184: the last turn DELIVERED and its count
    void update(int64_t t, int64_t c) {
        std::lock_guard<std::mutex> lk(mu);
        turn = t;
        count = c;
    }
    void halt() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
    }
};

// The ordered event stream of one Run: the turn loop hands each stepped chunk's results (and every
// other event, in order) to a delivery thread, which turns them into CellFlipped / TurnComplete
// events on `events` and latches the ticker, while the turn loop already steps the next chunk on the
// GPU -- device work of chunk n+1 overlaps the delivery of chunk n.  At most `depth` batches wait,
// so the turn loop runs at most that far ahead of what the consumer has seen (key latency).
class Pipeline {
public:
    struct Batch {
        int64_t turn0 = 0;                 // turns: completed turns before the chunk
        std::vector<uint64_t> alive;       // alive after each of the chunk's turns
        std::vector<uint64_t> per_turn;    // per-turn CellFlipped counts (flip events only)
        std::vector<int32_t> xy;           // every turn's flipped cells, turn by turn
        std::vector<Event> events;         // or: these events, as they are
        bool flips = false;
    };

    // depth 0: no delivery thread -- each batch is delivered by the turn loop itself before it
    // steps on (the unpipelined A/B: device work and event delivery alternate)
    Pipeline(Channel<Event> *events, Ticker *ticker, size_t depth)
        : events_(events), ticker_(ticker), q_(std::max<size_t>(depth, 1)), inline_(depth == 0) {
        if (!inline_) th_ = std::thread([this] { deliver(); });
    }
    ~Pipeline() {
        if (th_.joinable()) {  // unwinding: the consumer may not drain events any more
            q_.close();
            events_->close();
            th_.join();
        }
    }
    void turns(int64_t turn0, std::vector<uint64_t> &&alive) {
        Batch b;
        b.turn0 = turn0;
        b.alive = std::move(alive);
        push(std::move(b));
    }
    void flips(int64_t turn0, std::vector<uint64_t> &&alive, std::vector<uint64_t> &&per_turn,
               std::vector<int32_t> &&xy) {
        Batch b;
        b.turn0 = turn0;
        b.alive = std::move(alive);
        b.per_turn = std::move(per_turn);
        b.xy = std::move(xy);
        b.flips = true;
        push(std::move(b));
    }
    void event(Event e) {
        Batch b;
        b.events.push_back(std::move(e));
        push(std::move(b));
    }
    // every batch handed over so far has been delivered
    void finish() {
        q_.close();
        if (th_.joinable()) th_.join();
        if (failed_) std::rethrow_exception(failed_);
    }

private:
    void push(Batch &&b) {
        if (inline_) {
            deliver_batch(b);
            return;
        }
        try {
            q_.send(std::move(b));
        } catch (...) {  // closed by a failed delivery (failed_ was set before the close)
            if (failed_) std::rethrow_exception(failed_);
            throw;
        }
    }
    void deliver_batch(Batch &b) {
        if (!b.events.empty()) {
            events_->send_all(std::move(b.events));
            return;
        }
        std::vector<Event> out;
        size_t at = 0;
        // the ticker latches a turn once its TurnComplete is on its way (the reference latches on
        // turnChan, gol/distributor.go:180-184): deliver in slices so a tick never waits for a
        // whole chunk, and never reports a turn not yet delivered
        constexpr size_t kSlice = 4096;
        out.reserve(kSlice + 64);
        for (size_t i = 0; i < b.alive.size(); ++i) {
            const int64_t t = b.turn0 + (int64_t)i;  // the turn being computed
            if (b.flips)  // per turn: CellFlipped{turn} for each flipped cell, then TurnComplete
                for (uint64_t c = 0; c < b.per_turn[i]; ++c, ++at)
                    out.push_back(Event::cell_flipped(t, Cell{b.xy[2 * at], b.xy[2 * at + 1]}));
            out.push_back(Event::turn_complete(t + 1));
            if (out.size() >= kSlice || i + 1 == b.alive.size()) {
                events_->send_all(std::move(out));
                out.clear();
                ticker_->update(t + 1, (int64_t)b.alive[i]);
            }
        }
    }
    void deliver() {
        try {
            while (auto b = q_.recv()) deliver_batch(*b);
        } catch (...) {
            failed_ = std::current_exception();
            q_.close();
        }
    }

    Channel<Event> *events_;
    Ticker *ticker_;
    Channel<Batch> q_;
    bool inline_;
    std::thread th_;
    std::exception_ptr failed_;
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
    Pipeline pipe(events, &ticker, (size_t)std::max(1, o.pipeline_depth));

    bool quit = false;
    // Keys (gol/distributor.go:115-148), serviced between step chunks; their events go through the
    // pipeline, after every event of the turns before them
    auto handle_key = [&](char key, bool &paused) {
        switch (key) {
            case 's': {
                const std::string f = name + "x" + std::to_string(turn);
                snapshot(*eng, p, o, f);
                pipe.event(Event::image_output_complete(turn, f));
                break;
            }
            case 'q': {
                // Pause{P: true, Turn, Dimension} parks the state in the broker (:139-147): the
                // checkpoint file outlives this process; a later Run resumes from it
                eng->checkpoint_save(ckpt);
                pipe.event(Event::state_change(turn, State::Quitting));
                quit = true;
                break;
            }
            case 'k': {
                const std::string f = name + "x" + std::to_string(turn);
                snapshot(*eng, p, o, f);
                pipe.event(Event::image_output_complete(turn, f));
                pipe.event(Event::state_change(turn, State::Quitting));
                eng.reset();  // Broker.Quit -> GolOP.Quit: the workers go away
                reset_saved_state(o);
                quit = true;
                break;
            }
            case 'p':
                paused = !paused;
                pipe.event(Event::state_change(turn, paused ? State::Paused : State::Executing));
                break;
            default: break;
        }
    };

    // Chunks of turns: golhip_step with per-turn counts, or golhip_step_flips for per-turn
    // CellFlipped (each turn's flips kept in a device ring, one extraction per chunk).  Chunk sizes
    // grow while a chunk's device call takes less than chunk_seconds, so keys wait at most about
    // that long (plus the pipeline's queued chunks); the events of a chunk are delivered by the
    // pipeline while the next chunk runs.
    const int64_t ring_cap = o.flip_events ? eng->flips_ring_capacity() : 1;
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
            const int64_t n = std::min<int64_t>({chunk, p.Turns - turn, ring_cap});
            std::vector<int32_t> fxy;
            std::vector<uint64_t> fper, falive;
            eng->step_flips(n, fxy, fper, falive);
            pipe.flips(turn, std::move(falive), std::move(fper), std::move(fxy));
            turn += n;
        } else {
            const int64_t n = std::min<int64_t>(chunk, p.Turns - turn);
            pipe.turns(turn, eng->step(n, true));
            turn += n;
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt < o.chunk_seconds && chunk < (1 << 20)) chunk *= 2;
        if (dt > 4 * o.chunk_seconds && chunk > 1) chunk /= 2;
    }

    if (quit) {  // 'q' / 'k': FinalTurnComplete with no cells (gol/distributor.go:128,147)
        pipe.finish();
        ticker.halt();
        events->send(Event::final_turn_complete(turn, {}));
        events->close();
        return;
    }

    std::vector<Cell> alive = to_cells(eng->alive_cells());  // gol/distributor.go:235
    pipe.finish();
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
