// configs[0] call latency from C++ (no Python in the loop): golhip_step(h, 100, counts) on a
// 512^2 random board, wall time per call, and the same with counts off.
// Build: g++ -O2 -std=c++17 -Iinclude scripts/cfg0_call.cpp -Ldistributed-gol_amd/lib -lgolhip
//        -Wl,-rpath,$PWD/distributed-gol_amd/lib -o /tmp/cfg0_call
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>
#include "golhip.h"

int main() {
    golhip_t h = nullptr;
    if (golhip_create(512, 512, 1, 16, &h)) return 1;
    golhip_init_random(h, 5, 0x80000000u);
    std::vector<uint64_t> counts(100);
    for (int counting : {1, 0}) {
        for (int i = 0; i < 3; ++i) golhip_step(h, 100, counting ? counts.data() : nullptr);
        std::vector<double> us;
        for (int i = 0; i < 40; ++i) {
            golhip_sync(h);
            const auto t0 = std::chrono::steady_clock::now();
            if (golhip_step(h, 100, counting ? counts.data() : nullptr)) return 2;
            if (!counting) golhip_sync(h);
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(us.begin(), us.end());
        std::printf("counts=%d us per 100-turn call p10 %.1f p50 %.1f p90 %.1f\n", counting, us[4], us[20], us[36]);
    }
    golhip_destroy(h);
    return 0;
}
