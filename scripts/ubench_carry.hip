// ubench_carry.hip -- throughput of the lane-mask (SGPR) carry ops on gfx950, and of whole
// row-sum sequences built from them, cycles per wave64 instruction (or per word) per SIMD.
//
// Question: can the one-bit west shift of a packed row (c << 1 | west >> 31, west = lane - 1)
// be done with full-rate ops and a scalar lane-mask shift instead of DPP + v_alignbit (both
// measured at ~4 cycles, profiles/r01_ubench_valu2_clocked.txt)?
//   M  = ballot(c < 0)           v_cmp_gt_i32 -> SGPR pair   (bit 31 of every lane)
//   M1 = M << 1                  s_lshl_b64 (SALU)           (lane i gets lane i-1's bit)
//   h1 = c + c + M1[lane]        v_addc_co_u32 carry-in SGPR (= c << 1 | west >> 31)
// Same harness as ubench_valu2.hip: s_memtime/s_memrealtime, chip span over all waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define N_CHAIN 8
#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned long long *clk, unsigned seed) {
    unsigned v[N_CHAIN];
#pragma unroll
    for (int i = 0; i < N_CHAIN; ++i) v[i] = seed * (threadIdx.x + 1) + i * 977;
    unsigned a = seed ^ threadIdx.x, b = seed + blockIdx.x;
    unsigned long long msk = __builtin_amdgcn_ballot_w64((threadIdx.x & 3) == 1);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < N_CHAIN; ++i) {
            unsigned long long d;
            if (OP == 0) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "s"(msk));
            if (OP == 1) asm volatile("v_addc_co_u32_e64 %0, %1, %0, %0, %2" : "+v"(v[i]), "=s"(d) : "s"(msk));
            if (OP == 2) asm volatile("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(d) : "v"(v[i]));
            if (OP == 3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 4) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 5) asm volatile("v_bfe_u32 %0, %0, 30, 1" : "+v"(v[i]));
            if (OP == 6) asm volatile("v_add_co_u32_e64 %0, %1, %0, %0" : "+v"(v[i]), "=s"(d));
            if (OP == 7) {  // cmp -> s_lshl -> addc, one dependent chain per i
                asm volatile("v_cmp_gt_i32_e64 %1, 0, %0\n\ts_lshl_b64 %1, %1, 1\n\t"
                             "v_addc_co_u32_e64 %0, %2, %0, %0, %1"
                             : "+v"(v[i]), "=&s"(d), "=&s"(msk));
            }
            if (OP == 8) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(a));
            if (OP == 9) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(v[i]) :: "vcc");
            if (OP == 10) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            if (OP == 11) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            if (OP == 12) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1" :: "v"(v[i]), "v"(a) : "vcc");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = (unsigned)msk;
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

// Whole row-sum + rule step on R independent rows per lane, the two shift schemes:
//   SCHEME 0: w = dpp wave_shr:1 (c); h1 = alignbit(c, w, 31); h2 = alignbit(c, w, 30)
//   SCHEME 1: M = cmp(c<0); h1 = addc(c, c, M<<1); N = cmp(h1<0); h2 = addc(h1, h1, N<<1)
// then s0 = xor3(c,h1,h2), s1 = maj(c,h1,h2) and 7 more bitop3 (the vertical add + rule) that
// read the row sums of three rows. Reported per word (row) per generation.
template <int SCHEME>
__global__ __launch_bounds__(256) void rows(unsigned *out, unsigned long long *clk, unsigned seed) {
    constexpr int R = 6;
    unsigned c[R];
#pragma unroll
    for (int i = 0; i < R; ++i) c[i] = seed * (threadIdx.x + 7) + i * 12345;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS / 4; ++it) {
        unsigned s0[R], s1[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            unsigned h1, h2;
            if (SCHEME == 0) {
                unsigned w;
                asm("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                             : "=v"(w) : "v"(c[i]));
                h1 = __builtin_amdgcn_alignbit(c[i], w, 31);
                h2 = __builtin_amdgcn_alignbit(c[i], w, 30);
            } else {
                unsigned long long m, n, d0, d1;
                asm("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(m) : "v"(c[i]));
                m <<= 1;
                asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(h1), "=s"(d0) : "v"(c[i]), "s"(m));
                asm("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(n) : "v"(h1));
                n <<= 1;
                asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(h2), "=s"(d1) : "v"(h1), "s"(n));
            }
            s0[i] = __builtin_amdgcn_bitop3_b32(c[i], h1, h2, 0x96);
            s1[i] = __builtin_amdgcn_bitop3_b32(c[i], h1, h2, 0xe8);
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int u = (i + R - 1) % R, d = (i + 1) % R;
            // 7 bitop3 of the vertical add + rule shape (data-dependent on three rows)
            unsigned l0 = __builtin_amdgcn_bitop3_b32(s0[u], s0[i], s0[d], 0x96);
            unsigned k0 = __builtin_amdgcn_bitop3_b32(s0[u], s0[i], s0[d], 0xe8);
            unsigned x = __builtin_amdgcn_bitop3_b32(s1[u], s1[i], s1[d], 0x96);
            unsigned m = __builtin_amdgcn_bitop3_b32(s1[u], s1[i], s1[d], 0xe8);
            unsigned p = __builtin_amdgcn_bitop3_b32(x, k0, m, 0x14);
            unsigned q = __builtin_amdgcn_bitop3_b32(x, k0, m, 0x81);
            c[i] = __builtin_amdgcn_bitop3_b32(l0, p, q, 0xca) ^ 0;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) s ^= c[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[4 * wv] = t1 - t0;
        clk[4 * wv + 1] = r1 - r0;
        clk[4 * wv + 2] = r0;
        clk[4 * wv + 3] = r1;
    }
}

template <typename F>
void report(const char *name, double units, int wps, int blocks, unsigned long long *c, F launch) {
    launch();
    launch();
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(4 * blocks * 4);
    (void)hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    unsigned long long s0 = ~0ull, e1 = 0;
    for (int i = 0; i < blocks * 4; ++i) {
        cyc += h[4 * i]; real += h[4 * i + 1];
        s0 = std::min(s0, h[4 * i + 2]);
        e1 = std::max(e1, h[4 * i + 3]);
    }
    cyc /= blocks * 4; real /= blocks * 4;
    const double ghz = cyc / (real * 10.0);
    const double span_cyc = (double)(e1 - s0) * 10.0 * ghz;
    std::printf("%-34s w/SIMD %d: chip-span %.2f cyc/unit/SIMD; %.2f GHz\n", name, wps,
                span_cyc / (units * wps), ghz);
}

template <int OP>
void run(const char *name, int ipc, unsigned *d, unsigned long long *c, int wps) {
    const int blocks = 256 * wps;
    report(name, (double)ITERS * N_CHAIN * ipc, wps, blocks, c,
           [&] { hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, c, 1u); });
}

template <int S>
void run_rows(const char *name, unsigned *d, unsigned long long *c, int wps) {
    const int blocks = 256 * wps;
    report(name, (double)(ITERS / 4) * 6, wps, blocks, c,
           [&] { hipLaunchKernelGGL(rows<S>, dim3(blocks), dim3(256), 0, 0, d, c, 1u); });
}

int main() {
    unsigned *d; unsigned long long *c;
    (void)hipMalloc(&d, 256 * 8 * 256 * 4);
    (void)hipMalloc(&c, 256 * 8 * 4 * 32);
    for (int w : {2, 4}) {
        run<10>("v_sub_u32 (reference, full rate)", 1, d, c, w);
        run<0>("v_cndmask_b32_e64 sgpr mask", 1, d, c, w);
        run<8>("v_cndmask_b32_e32 vcc", 1, d, c, w);
        run<1>("v_addc_co_u32_e64 sgpr carry", 1, d, c, w);
        run<9>("v_addc_co_u32_e32 vcc", 1, d, c, w);
        run<2>("v_cmp_gt_i32_e64 -> sgpr", 1, d, c, w);
        run<12>("v_cmp_eq_u32_e32 -> vcc", 1, d, c, w);
        run<6>("v_add_co_u32_e64 carry-out", 1, d, c, w);
        run<3>("v_add3_u32", 1, d, c, w);
        run<11>("v_or3_b32", 1, d, c, w);
        run<4>("v_lshl_add_u32", 1, d, c, w);
        run<5>("v_bfe_u32", 1, d, c, w);
        run<7>("cmp+s_lshl+addc (per triple)", 1, d, c, w);
        run_rows<0>("rows: dpp + 2 alignbit + 9 bitop3", d, c, w);
        run_rows<1>("rows: 2x(cmp,s_lshl,addc) + 9 bitop3", d, c, w);
    }
    return 0;
}
