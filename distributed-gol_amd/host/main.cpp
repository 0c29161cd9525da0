// main.cpp -- headless CLI mirroring the reference's main.go:13-68 flags on the C++ host.
//   -t threads  -w width  -h height  -turns N  -noVis (always headless: SDL is out of scope)
//   extra: -gpus G (row strips), -k K (max generations per launch), -images DIR, -out DIR,
//          -checkpoint PATH (the 'q' state file; default OUT/broker_state.ckpt), -flips
// Keys p/s/q/k are read from stdin (one character per line), like the SDL key loop
// (sdl/loop.go:17-27) would deliver them.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>

#include "gol.hpp"

int main(int argc, char **argv) {
    gol::Params p{10000000000LL, 8, 512, 512};  // main.go:38-42 defaults: 8 threads, 512x512, 1e10 turns
    gol::RunOptions o;
    o.flip_events = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : "0"; };
        if (a == "-t") p.Threads = std::atoi(next());
        else if (a == "-w") p.ImageWidth = std::atoi(next());
        else if (a == "-h") p.ImageHeight = std::atoi(next());
        else if (a == "-turns") p.Turns = std::strtoll(next(), nullptr, 10);  // Go int: 64-bit
        else if (a == "-gpus") o.ngpus = std::atoi(next());
        else if (a == "-k") o.k = std::atoi(next());
        else if (a == "-images") o.image_dir = next();
        else if (a == "-out") o.out_dir = next();
        else if (a == "-checkpoint") o.checkpoint_path = next();
        else if (a == "-flips") o.flip_events = true;
        else if (a == "-noVis") {}
    }
    std::printf("Threads: %d\nWidth: %d\nHeight: %d\n", p.Threads, p.ImageWidth, p.ImageHeight);
    gol::Channel<gol::Event> events(1000);  // main.go:210
    gol::Channel<char> keys(10);            // main.go:209
    std::thread keyreader([&] {
        std::string line;
        while (std::getline(std::cin, line))
            if (!line.empty()) {
                try { keys.send(line[0]); } catch (...) { return; }
            }
    });
    keyreader.detach();
    std::thread run([&] { gol::Run(p, &events, &keys, o); });
    while (auto e = events.recv()) {
        const std::string s = e->String();
        if (!s.empty())
            std::printf("Completed Turns %-8lld%s\n", (long long)e->GetCompletedTurns(), s.c_str());
        if (e->kind == gol::EventKind::FinalTurnComplete)
            std::printf("Final turn %lld: %zu alive cells\n", (long long)e->CompletedTurns,
                        e->Alive->size());
    }
    run.join();
    std::fflush(stdout);
    std::_Exit(0);  // the key reader may still block on stdin
}
