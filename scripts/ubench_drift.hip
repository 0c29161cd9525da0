// ubench_drift.hip -- the VALU issue ceiling of the production level update, measured without
// memory: the drifting-sum update of gol_stencil (1 DPP + 2 v_alignbit + 2 v_bitop3 for the row's
// 3-cell sums, 7 v_bitop3 for B3/S23 -- golhip_stencil.hpp row_sum3_drift / life_next) chained
// over K = 14 levels per step, like the production K = 14 launch, on every SIMD of the chip at 4
// waves per SIMD, fed with random rows (a dense board's bit activity) or zero rows (no toggles).
// Reports the wave64 VALU instructions per second the chip issues for this exact mix, the
// in-kernel shader clock (s_memtime / s_memrealtime) and cycles per instruction per SIMD -- the
// ceiling the production kernel's issued rate (PMC SQ_INSTS_VALU / duration) is compared with.
// Usage: ubench_drift [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define GOL_TT(EXPR) ((uint8_t)([](uint32_t a, uint32_t b, uint32_t c) { return (EXPR); }(0xF0u, 0xCCu, 0xAAu)))
#define GOL_BOP3(A, B, C, TT) __builtin_amdgcn_bitop3_b32((A), (B), (C), (TT))
constexpr uint8_t kXor3 = GOL_TT(a ^ b ^ c);
constexpr uint8_t kMaj = GOL_TT((a & b) | (c & (a | b)));
constexpr uint8_t kTwosEven = GOL_TT(~(a | b | c) | (~a & ~b & c) | (a & b & ~c));
constexpr uint8_t kOddSelect = GOL_TT((a & ~b) | (~a & c));

constexpr int K = 14;      // levels per step (the production bulk depth at 65536^2)
constexpr int STEPS = 8;   // steps per loop iteration (input rows cycled from registers)
constexpr int ITERS = 2000;

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

struct Level {
    uint32_t as, acy, ms, mcy, mc;
};

template <bool RANDOM>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned long long *clk, unsigned seed) {
    const unsigned tid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t z = seed >> 31;  // 0 at run time (seed < 2^31), unknown to the compiler
    uint32_t rows[STEPS];
#pragma unroll
    for (int i = 0; i < STEPS; ++i) rows[i] = RANDOM ? hash32(tid * 131 + i + seed) : z;
    Level L[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        L[j].as = RANDOM ? hash32(tid * 7 + j) : z;
        L[j].acy = RANDOM ? hash32(tid * 11 + j) : z;
        L[j].ms = RANDOM ? hash32(tid * 13 + j) : z;
        L[j].mcy = RANDOM ? hash32(tid * 17 + j) : z;
        L[j].mc = RANDOM ? hash32(tid * 19 + j) : z;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int st = 0; st < STEPS; ++st) {
            uint32_t in = rows[st] ^ acc;  // the new input row of level 0 (1 extra op per step)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                // row_sum3_drift: only the WEST neighbour word (one DPP), two funnel shifts
                const uint32_t wl = (uint32_t)__builtin_amdgcn_mov_dpp((int)in, 0x138, 0xf, 0xf, false);
                const uint32_t w1 = __builtin_amdgcn_alignbit(in, wl, 31);
                const uint32_t w2 = __builtin_amdgcn_alignbit(in, wl, 30);
                const uint32_t ns = GOL_BOP3(w2, w1, in, kXor3);
                const uint32_t ncy = GOL_BOP3(w2, w1, in, kMaj);
                // life_next of the level's middle row (7 v_bitop3)
                const uint32_t o = GOL_BOP3(L[j].as, L[j].ms, ns, kXor3);
                const uint32_t kk = GOL_BOP3(L[j].as, L[j].ms, ns, kMaj);
                const uint32_t p = GOL_BOP3(L[j].acy, L[j].mcy, ncy, kXor3);
                const uint32_t q = GOL_BOP3(L[j].acy, L[j].mcy, ncy, kMaj);
                const uint32_t u = GOL_BOP3(kk, p, q, kTwosEven);
                const uint32_t v = GOL_BOP3(o, q, L[j].mc, kOddSelect);
                const uint32_t nx = GOL_BOP3(v, o, u, GOL_TT(a & (b ^ c)));
                L[j].as = L[j].ms, L[j].acy = L[j].mcy;
                L[j].ms = ns, L[j].mcy = ncy, L[j].mc = w1;
                in = nx;  // the next level's input row
            }
            acc = in;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[tid] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 4;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 4;  // 4 blocks of 4 waves per CU: 4 waves per SIMD (production K = 14)
    unsigned *out;
    unsigned long long *clk;
    (void)hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    (void)hipMalloc(&clk, sizeof(unsigned long long) * 2 * blocks);
    std::vector<unsigned long long> h(2 * blocks);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    (void)hipDeviceSynchronize();
    const double instr_per_wave = (double)ITERS * STEPS * (K * 12 + 1);
    const double waves = (double)blocks * 4;
    printf("{\"cus\": %d, \"waves_per_simd\": 4, \"levels\": %d, \"valu_per_level_update\": 12, \"runs\": [", cus, K);
    for (int r = 0; r < 2 * reps; ++r) {
        const bool rnd = (r % 2) == 0;
        (void)hipEventRecord(e0, 0);
        if (rnd) hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u + r);
        else hipLaunchKernelGGL(k<false>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u + r);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
        std::vector<double> ghz;
        for (int b = 0; b < blocks; ++b) ghz.push_back((double)h[2 * b] / ((double)h[2 * b + 1] * 10.0));
        std::sort(ghz.begin(), ghz.end());
        const double clock = ghz[ghz.size() / 2];
        const double tinstr = waves * instr_per_wave / (ms * 1e-3) / 1e12;
        const double cyc = (ms * 1e-3) * clock * 1e9 / (instr_per_wave * 4);  // per instruction per SIMD
        printf("%s{\"data\": \"%s\", \"ms\": %.3f, \"t_instr_per_s\": %.4f, \"clock_ghz\": %.3f, "
               "\"cycles_per_instr_per_simd\": %.3f}",
               r ? ", " : "", rnd ? "random" : "zero", ms, tinstr, clock, cyc);
    }
    printf("]}\n");
    return 0;
}
