// ubench_valu2.hip -- cycles per wave64 VALU instruction per SIMD on gfx950, measured in-kernel
// with s_memtime (shader clock) and s_memrealtime (100 MHz), at W waves per SIMD.
// Each lane runs 16 independent chains; the per-SIMD throughput = W waves * instrs / cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define N_CHAIN 16
#define ITERS 8192

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned long long *clk, unsigned seed) {
    unsigned v[N_CHAIN];
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) v[i] = seed * (threadIdx.x + 1) + i * 977;
    unsigned a = seed ^ threadIdx.x, b = seed + blockIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < N_CHAIN; ++i) {
            if (OP == 0) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[i]) : "v"(a));
            if (OP == 2) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
            if (OP == 3) asm volatile("v_or_b32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]) : "v"(a));
            if (OP == 4) { unsigned long long x = ((unsigned long long)v[i] << 32) | a;
                           asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x)); v[i] = (unsigned)(x >> 32); }
            if (OP == 5) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 6) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 7) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(v[i]));
            if (OP == 8) asm volatile("v_add_u32 %0, %0, %0" : "+v"(v[i]));
            if (OP == 9) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 10) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 11) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(v[i]));
            if (OP == 12) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(a));
            if (OP == 13) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(v[i]));
            if (OP == 14) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b));
                            asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[(i + 8) % N_CHAIN]) : "v"(a)); }
            if (OP == 15) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 16) asm volatile("v_mov_b32_sdwa %0, %0 dst_sel:DWORD src0_sel:WORD_1" : "+v"(v[i]));
            if (OP == 17) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            // pairs: cross-lane op + bitop3
            if (OP == 18) { asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)); }
            if (OP == 19) { unsigned t; asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(t) : "v"(v[i]));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(t), "v"(b)); }
            if (OP == 20) { unsigned t; asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(t) : "v"(v[(i + 8) % N_CHAIN]));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(t), "v"(b)); }
            if (OP == 21) { asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)); }
            if (OP == 22) { asm volatile("v_mov_b32_e32 %0, %0" : "+v"(v[i]));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)); }
            if (OP == 23) { asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[i]) : "v"(a));
                            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)); }
            if (OP == 24) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i+1)%N_CHAIN]), "v"(v[(i+2)%N_CHAIN])); }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) s ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[4 * wv] = t1 - t0;
        clk[4 * wv + 1] = r1 - r0;
        clk[4 * wv + 2] = r0;
        clk[4 * wv + 3] = r1;
    }
}

template <int OP>
void run(const char *name, int ipc, unsigned *d, unsigned long long *c, int wps) {
    const int blocks = 256 * wps;  // 4-wave blocks: wps blocks per CU = wps waves per SIMD
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, c, 1u);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, c, 1u);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(4 * blocks * 4);
    hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
    for (int i = 0; i < blocks * 4; ++i) {
        cyc += h[4 * i]; real += h[4 * i + 1];
        s0 = std::min(s0, h[4 * i + 2]); s1 = std::max(s1, h[4 * i + 2]);
        e0 = std::min(e0, h[4 * i + 3]); e1 = std::max(e1, h[4 * i + 3]);
    }
    cyc /= blocks * 4; real /= blocks * 4;
    const double ghz = cyc / (real * 10.0);
    const double instr = (double)ITERS * N_CHAIN * ipc;
    // chip-level: every SIMD ran wps waves; span = first start .. last end (realtime, 100 MHz)
    const double span_cyc = (double)(e1 - s0) * 10.0 * ghz;
    std::printf("%-24s w/SIMD %d: per-wave %.2f, chip-span %.2f cyc/instr/SIMD; %.2f GHz; start spread %.1f%%, end spread %.1f%% of span\n",
                name, wps, cyc / (instr * wps), span_cyc / (instr * wps), ghz,
                100.0 * (s1 - s0) / (e1 - s0), 100.0 * (e1 - e0) / (e1 - s0));
}

int main() {
    unsigned *d; unsigned long long *c;
    hipMalloc(&d, 256 * 8 * 256 * 4); hipMalloc(&c, 256 * 8 * 4 * 32);
    for (int w : {4, 8}) {
        run<18>("pair dpp(x),bitop3(x)", 2, d, c, w);
        run<19>("pair dpp(x)->t,bitop3(x,t)", 2, d, c, w);
        run<20>("pair dpp(other),bitop3", 2, d, c, w);
        run<21>("pair dpp row_shr,bitop3", 2, d, c, w);
        run<22>("pair mov,bitop3", 2, d, c, w);
        run<23>("pair alignbit,bitop3", 2, d, c, w);
        run<24>("bitop3 3 vgpr srcs", 1, d, c, w);
    }
    for (int w : {4}) {
        run<0>("v_bitop3_b32", 1, d, c, w);
        run<1>("v_alignbit_b32", 1, d, c, w);
        run<2>("v_mov_b32_dpp wave_shr", 1, d, c, w);
        run<13>("v_mov_b32_dpp row_shr", 1, d, c, w);
        run<3>("v_or_b32_dpp wave_shr", 1, d, c, w);
        run<4>("v_lshlrev_b64", 1, d, c, w);
        run<5>("v_lshl_or_b32", 1, d, c, w);
        run<6>("v_xor_b32", 1, d, c, w);
        run<17>("v_and_b32", 1, d, c, w);
        run<7>("v_lshrrev_b32", 1, d, c, w);
        run<8>("v_add_u32", 1, d, c, w);
        run<9>("v_perm_b32", 1, d, c, w);
        run<10>("v_bcnt_u32_b32", 1, d, c, w);
        run<11>("v_lshlrev_b32", 1, d, c, w);
        run<12>("v_cndmask_b32", 1, d, c, w);
        run<14>("bitop3+alignbit pair", 2, d, c, w);
        run<15>("v_pk_add_u16", 1, d, c, w);
        run<16>("v_mov_b32_sdwa", 1, d, c, w);
    }
    return 0;
}
