// ubench_valu.hip -- VALU throughput of the instructions the stencil is made of, on gfx950.
// 16 independent dependency chains per lane, 8 waves per SIMD; reports cycles per wave64
// instruction per SIMD (clock from s_memtime would need a diagnostic build; we report ns and
// derive cycles at the measured kernel clock via GRBM in rocprof if wanted).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

#define N_CHAIN 16
#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned seed) {
    unsigned v[N_CHAIN];
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) v[i] = seed * (threadIdx.x + 1) + i * 977;
    unsigned a = seed ^ threadIdx.x, b = seed + blockIdx.x;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < N_CHAIN; ++i) {
            if (OP == 0) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[i]) : "v"(a));
            if (OP == 3) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
            if (OP == 4) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
            if (OP == 5) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 6) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 7) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
        }
    }
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) s ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
double run(unsigned *d, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    unsigned *d; hipMalloc(&d, blocks * 256 * 4);
    const char *names[] = {"v_bitop3_b32", "v_xor_b32", "v_alignbit_b32", "v_mov_dpp wave_shr",
                           "v_mov_dpp row_shr", "v_bfi_b32", "and_or", "bcnt+add"};
    double t[8];
    t[0] = run<0>(d, blocks); t[1] = run<1>(d, blocks); t[2] = run<2>(d, blocks); t[3] = run<3>(d, blocks);
    t[4] = run<4>(d, blocks); t[5] = run<5>(d, blocks); t[6] = run<6>(d, blocks); t[7] = run<7>(d, blocks);
    const double waves = blocks * 4.0, ops = waves * ITERS * N_CHAIN;  // wave-instructions
    for (int i = 0; i < 8; ++i) {
        // wave-instructions per SIMD per ns
        const double per_simd_ns = t[i] * 1e6 / (ops / 1024.0);
        std::printf("%-22s %8.3f ms  %.3f ns per wave-instr per SIMD (= %.2f cycles at 2.2 GHz)\n",
                    names[i], t[i], per_simd_ns, per_simd_ns * 2.2);
    }
    return 0;
}
