// ubench_toggle.hip -- does the chip's VALU throughput depend on the DATA? The same v_bitop3
// (XOR3) stream over the whole chip (4 waves per SIMD, 16 independent chains per lane), either on
// random operands (about half the bits of every result toggle each instruction, like the stencil
// on a dense board) or on zero operands (nothing toggles).  Reports, per mode, the wall time, the
// shader clock measured in-kernel (s_memtime over s_memrealtime at 100 MHz) and the cycles per
// wave64 instruction per SIMD.  Usage: ubench_toggle [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define N_CHAIN 16
#define ITERS 100000

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <bool RANDOM>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned long long *clk, unsigned seed) {
    const unsigned tid = blockIdx.x * 256 + threadIdx.x;
    unsigned v[N_CHAIN], a[N_CHAIN];
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) {
        v[i] = RANDOM ? hash32(tid * 131 + i + seed) : 0u;
        a[i] = RANDOM ? hash32(tid * 977 + i * 7 + seed * 3) : 0u;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < N_CHAIN; ++i)  // v ^= a ^ a': with random a, ~half the bits flip
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a[i]), "v"(a[(i + 5) % N_CHAIN]));
#pragma unroll
        for (int i = 0; i < N_CHAIN; ++i)
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a[(i + 3) % N_CHAIN]), "v"(a[(i + 11) % N_CHAIN]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) x ^= v[i];
    out[tid] = x;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 4;  // 4 blocks of 4 waves per CU: 4 waves per SIMD
    unsigned *out;
    unsigned long long *clk;
    hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipMalloc(&clk, sizeof(unsigned long long) * 2 * blocks);
    std::vector<unsigned long long> h(2 * blocks);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // warm (and pre-heat the clock)
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    hipDeviceSynchronize();
    printf("{\"cus\": %d, \"waves_per_simd\": 4, \"instr_per_wave\": %d, \"runs\": [", cus, 2 * N_CHAIN * ITERS);
    for (int r = 0; r < 2 * reps; ++r) {
        const bool rnd = (r % 2) == 0;
        hipEventRecord(e0, 0);
        if (rnd) hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u + r);
        else hipLaunchKernelGGL(k<false>, dim3(blocks), dim3(256), 0, 0, out, clk, 7u + r);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
        double ghz = 0;
        for (int b = 0; b < blocks; ++b) ghz += (double)h[2 * b] / ((double)h[2 * b + 1] / 100e6) / 1e9;
        ghz /= blocks;
        // wave64 instructions per SIMD / (time x clock) -> cycles per instruction per SIMD
        const double instr_per_simd = 4.0 * 2 * N_CHAIN * ITERS;
        const double cpi = (ms * 1e-3) * ghz * 1e9 / instr_per_simd;
        printf("%s{\"data\": \"%s\", \"ms\": %.3f, \"shader_ghz\": %.3f, \"cycles_per_valu_per_simd\": %.3f}",
               r ? ", " : "", rnd ? "random" : "zero", ms, ghz, cpi);
    }
    printf("]}\n");
    return 0;
}
