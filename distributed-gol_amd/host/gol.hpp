// gol.hpp -- C++ host mirror of the reference's public contract (package gol):
//
//   Params                      gol/gol.go:6-11
//   Run(p, events, keyPresses)  gol/gol.go:14-57   (distributor: gol/distributor.go:194-263)
//   Event + event kinds         gol/event.go:9-68  (String / GetCompletedTurns)
//   util.Cell                   util/cell.go:4-6
//   stubs Request / Response    stubs/stubs.go:15-29 (kept as value types for callers that
//                               speak the broker protocol; the engine answers Publish in-process)
//
// The reference is Go; there is no Go toolchain on this image, so the host side above the C ABI
// (include/golhip.h) is C++ (see INTEGRATION.md for the cgo binding a Go maintainer would add).
// Run() drives libgolhip instead of dialling the broker (gol/distributor.go:218-222): the board
// stays in HBM and the turn loop calls golhip_step in chunks so that the 2 s AliveCellsCount
// ticker and the p/s/q/k keys are serviced between chunks.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "channel.hpp"

namespace gol {

// util/cell.go:4-6
struct Cell {
    int X = 0, Y = 0;
    bool operator==(const Cell &o) const { return X == o.X && Y == o.Y; }
    bool operator<(const Cell &o) const { return Y != o.Y ? Y < o.Y : X < o.X; }
};

// gol/gol.go:6-11 (Go's int is 64-bit: Turns defaults to 1e10 in main.go:38-42)
struct Params {
    int64_t Turns = 0;
    int Threads = 1;  // kept for contract parity; the GPU grid replaces goroutine strips
    int ImageWidth = 0;
    int ImageHeight = 0;
};

// gol/event.go:32-38
enum class State { Paused, Executing, Quitting };
std::string to_string(State s);

// gol/event.go:19-68 -- one tagged struct instead of Go's interface of value types.
enum class EventKind {
    AliveCellsCount,      // CompletedTurns, CellsCount
    ImageOutputComplete,  // CompletedTurns, Filename
    StateChange,          // CompletedTurns, NewState
    CellFlipped,          // CompletedTurns, Cell
    TurnComplete,         // CompletedTurns
    FinalTurnComplete,    // CompletedTurns, Alive
};

struct Event {
    EventKind kind = EventKind::TurnComplete;
    int64_t CompletedTurns = 0;  // Go int
    int64_t CellsCount = 0;
    std::string Filename;
    State NewState = State::Executing;
    Cell cell;
    std::shared_ptr<std::vector<Cell>> Alive;  // FinalTurnComplete only
    // AliveCellsCount only, a host-mirror extra (no gol/event.go field): steady_clock ns at which
    // the ticker fired, so a consumer can measure tick latency (fire -> received)
    int64_t FiredNs = 0;

    // gol/event.go:71-131: the GUI prints events whose String() is non-empty (sdl/loop.go:44-47)
    std::string String() const;
    int64_t GetCompletedTurns() const { return CompletedTurns; }

    static Event alive_cells_count(int64_t turns, int64_t n);
    static Event image_output_complete(int64_t turns, std::string f);
    static Event state_change(int64_t turns, State s);
    static Event cell_flipped(int64_t turns, Cell c);
    static Event turn_complete(int64_t turns);
    static Event final_turn_complete(int64_t turns, std::vector<Cell> alive);
};

// stubs/stubs.go:15-29 (the broker wire types; World rows of 0/255 bytes)
struct Request {
    std::vector<std::vector<uint8_t>> World;
    int ImageSize = 0, SplitSize = 0, StartY = 0, EndY = 0, Threads = 0;
};
struct Response {
    std::vector<std::vector<uint8_t>> World;
    int Turn = 0;
    std::vector<Cell> FlipCells;
    std::vector<std::vector<uint8_t>> InitialWorld;
};

// Engine-side options (no reference equivalent; defaults reproduce the reference's behaviour).
struct RunOptions {
    std::string image_dir = "images";  // gol/io.go:96  images/<W>x<H>.pgm
    std::string out_dir = "out";       // gol/io.go:43  out/<name>.pgm
    int ngpus = 1;                     // row strips over this many GPUs
    int k = 8;                         // temporal-blocking depth when no per-turn flips are needed
    bool flip_events = true;           // per-turn CellFlipped (gol/distributor.go:53-59)
    int ticker_ms = 2000;              // AliveCellsCount period (gol/distributor.go:228)
    double chunk_seconds = 0.02;       // target device time per step chunk (key/ticker latency)
    // stepped chunks whose events may wait for delivery by the delivery thread while the turn
    // loop steps on (0: no delivery thread, device work and event delivery alternate)
    int pipeline_depth = 2;
    // The broker's paused state (worldSave, turn, size; broker/broker.go:124-155) as a file: 'q'
    // writes it, the next Run with Turns > 0 consumes it (CheckStates) and resumes when the size
    // matches.  Empty: <out_dir>/broker_state.ckpt.
    std::string checkpoint_path;
};

// gol/gol.go:14 -- runs the whole simulation, sends events, closes `events` at the end.
// keyPresses may be null (the tests pass nil, gol_test.go:34).
void Run(Params p, Channel<Event> *events, Channel<char> *keyPresses,
         const RunOptions &opts = RunOptions());

// Broker.Publish equivalent (broker/broker.go:157-180): one turn of req.World on the GPU.
// res.InitialWorld = req.World, res.World = next generation.
int Publish(const Request &req, Response *res, int ngpus = 1);

// Forget a board saved by 'q' (broker/broker.go:124-141 CheckStates clears `paused`).
void reset_saved_state(const RunOptions &opts = RunOptions());
std::string checkpoint_file(const RunOptions &opts);

// gol/io.go helpers (P5, maxval 255).
struct Image {
    int width = 0, height = 0;
    std::vector<uint8_t> pixels;  // row-major, width*height
};
Image read_pgm(const std::string &path);                       // gol/io.go:90-128
void write_pgm(const std::string &path, const Image &img);     // gol/io.go:42-87
std::vector<Cell> alive_cells_of(const Image &img);            // gol/distributor.go:153-166

}  // namespace gol
