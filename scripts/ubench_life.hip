// ubench_life.hip -- register-only throughput of the stencil's level update on gfx950 (no memory
// traffic): K chained levels per step, D words per lane, W waves per SIMD; reports cycles per
// wave-level-step per SIMD (chip span, shader clock from s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define GOL_TT(EXPR) ((uint8_t)([](uint32_t a, uint32_t b, uint32_t c) { return (EXPR); }(0xF0u, 0xCCu, 0xAAu)))
#define GOL_BOP3(A, B, C, TT) __builtin_amdgcn_bitop3_b32((A), (B), (C), (TT))
constexpr uint8_t kXor3 = GOL_TT(a ^ b ^ c);
constexpr uint8_t kMaj = GOL_TT((a & b) | (c & (a | b)));
constexpr uint8_t kTwosEven = GOL_TT(~(a | b | c) | (~a & ~b & c) | (a & b & ~c));
constexpr uint8_t kOddSelect = GOL_TT((a & ~b) | (~a & c));

template <int MODE>
__device__ __forceinline__ uint32_t xl(uint32_t v, int dir) {
    if (MODE == 1) return v ^ 0x5a5a5a5au;  // no cross-lane: plain full-rate op instead of DPP
    if (MODE == 3) {  // ds_bpermute (LDS crossbar)
        const int lane = __lane_id();
        const int src = dir ? ((lane + 1) & 63) : ((lane - 1) & 63);
        return (uint32_t)__builtin_amdgcn_ds_bpermute(src * 4, (int)v);
    }
    if (MODE == 4)
        return dir ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xf, 0xf, false)   // row_shl:1
                   : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    if (MODE == 5)  // DPP fused into a VOP2 op (v_xor_b32_dpp): cost of DPP as a modifier
        return dir ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false) ^ v
                   : (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false) ^ v;
    return dir ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, false)
               : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, false);
}

template <int D>
struct Words { uint32_t w[D]; };

template <int D, int MODE>
__device__ __forceinline__ void row_sum3(const Words<D> &c, Words<D> &s, Words<D> &cy) {
    const uint32_t wl = xl<MODE>(c.w[D - 1], 0);
    const uint32_t el = xl<MODE>(c.w[0], 1);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t left = d == 0 ? wl : c.w[d - 1];
        const uint32_t right = d == D - 1 ? el : c.w[d + 1];
        uint32_t w, e;
        if (MODE == 2) { w = left ^ c.w[d]; e = right ^ c.w[d]; }   // no shifts
        else { w = __builtin_amdgcn_alignbit(c.w[d], left, 31); e = __builtin_amdgcn_alignbit(right, c.w[d], 1); }
        s.w[d] = GOL_BOP3(w, c.w[d], e, kXor3);
        cy.w[d] = GOL_BOP3(w, c.w[d], e, kMaj);
    }
}

__device__ __forceinline__ uint32_t life_next(uint32_t as, uint32_t acy, uint32_t ms, uint32_t mcy,
                                              uint32_t mc, uint32_t bs, uint32_t bcy) {
    const uint32_t o = GOL_BOP3(as, ms, bs, kXor3);
    const uint32_t k = GOL_BOP3(as, ms, bs, kMaj);
    const uint32_t p = GOL_BOP3(acy, mcy, bcy, kXor3);
    const uint32_t q = GOL_BOP3(acy, mcy, bcy, kMaj);
    const uint32_t u = GOL_BOP3(k, p, q, kTwosEven);
    const uint32_t v = GOL_BOP3(o, q, mc, kOddSelect);
    return GOL_BOP3(v, o, u, GOL_TT(a & (b ^ c)));
}

template <int D> struct RowState { Words<D> s, cy, c; };

template <int D, int MODE>
__device__ __forceinline__ void level_update(RowState<D> &above, const RowState<D> &mid,
                                             const Words<D> &in, Words<D> &nx) {
    Words<D> ns, ncy;
    row_sum3<D, MODE>(in, ns, ncy);
#pragma unroll
    for (int d = 0; d < D; ++d)
        nx.w[d] = life_next(above.s.w[d], above.cy.w[d], mid.s.w[d], mid.cy.w[d], mid.c.w[d], ns.w[d], ncy.w[d]);
    above.s = ns; above.cy = ncy; above.c = in;
}

template <int K, int D, int MODE, int SKEW>
__global__ __launch_bounds__(256) void kern(uint32_t *out, unsigned long long *clk, int steps, uint32_t seed) {
    RowState<D> X[K], Y[K];
    Words<D> pend[K];
    const uint32_t lane = threadIdx.x;
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int d = 0; d < D; ++d) {
            X[j].s.w[d] = X[j].cy.w[d] = X[j].c.w[d] = lane * (j + 3) + d;
            Y[j].s.w[d] = Y[j].cy.w[d] = Y[j].c.w[d] = lane ^ (j * 77 + d);
            pend[j].w[d] = lane + j;
        }
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    auto step = [&](auto par, uint32_t sv) {
        constexpr int PAR = decltype(par)::value;
        Words<D> nc;
#pragma unroll
        for (int d = 0; d < D; ++d) nc.w[d] = sv * 0x9E3779B9u + lane + d;
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
            const int j = SKEW ? K - 1 - jj : jj;
            Words<D> lin = SKEW ? (j == 0 ? nc : pend[j]) : nc;
            Words<D> nx;
            if (PAR == 0) level_update<D, MODE>(X[j], Y[j], lin, nx);
            else level_update<D, MODE>(Y[j], X[j], lin, nx);
            if (j == K - 1) { acc += nx.w[0]; }
            else if (SKEW) pend[j + 1] = nx;
            else nc = nx;
        }
    };
    for (int s = 0; s < steps; s += 2) {
        step(std::integral_constant<int, 0>{}, (uint32_t)s ^ seed);
        step(std::integral_constant<int, 1>{}, (uint32_t)s + 1);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[4 * wv] = t1 - t0; clk[4 * wv + 1] = r1 - r0; clk[4 * wv + 2] = r0; clk[4 * wv + 3] = r1;
    }
}

template <int K, int D, int MODE, int SKEW>
void run(const char *name, int wps, uint32_t *d, unsigned long long *c) {
    const int blocks = 256 * wps, steps = 4096;
    auto f = kern<K, D, MODE, SKEW>;
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, f, 256, 0);
    if (occ < wps) { std::printf("%-28s K=%2d D=%d w/SIMD %d: skipped (occupancy %d)\n", name, K, D, wps, occ); return; }
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, steps, 1u);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, steps, 1u);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(4 * blocks * 4);
    hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    unsigned long long s0 = ~0ull, e1 = 0;
    for (int i = 0; i < blocks * 4; ++i) {
        cyc += h[4 * i]; real += h[4 * i + 1];
        s0 = std::min(s0, h[4 * i + 2]); e1 = std::max(e1, h[4 * i + 3]);
    }
    const double ghz = cyc / (real * 10.0);
    const double span = (double)(e1 - s0) * 10.0 * ghz;
    const double level_steps = (double)steps * K * D * wps;  // word-level-steps per SIMD
    std::printf("%-28s K=%2d D=%d w/SIMD %d: %.2f cycles per word-level per SIMD (%.2f GHz)\n", name, K, D, wps,
                span / level_steps, ghz);
}

int main() {
    uint32_t *d; unsigned long long *c;
    hipMalloc(&d, 256 * 8 * 256 * 4); hipMalloc(&c, 256 * 8 * 4 * 32);
    for (int w : {2, 4, 8}) {
        run<8, 1, 3, 0>("chain bpermute", w, d, c);
        run<8, 1, 4, 0>("chain dpp row_shr", w, d, c);
        run<8, 1, 5, 0>("chain dpp+xor", w, d, c);
        run<8, 1, 3, 1>("skew bpermute", w, d, c);
        run<4, 2, 3, 0>("chain bpermute", w, d, c);
        run<8, 1, 0, 0>("chain full", w, d, c);
        run<8, 1, 1, 0>("chain no-DPP", w, d, c);
        run<8, 1, 2, 0>("chain no-shift", w, d, c);
        run<8, 1, 0, 1>("skew full", w, d, c);
        run<16, 1, 0, 0>("chain full", w, d, c);
        run<16, 1, 0, 1>("skew full", w, d, c);
        run<8, 2, 0, 0>("chain full", w, d, c);
        run<8, 2, 0, 1>("skew full", w, d, c);
        run<4, 2, 0, 0>("chain full", w, d, c);
        run<4, 1, 0, 0>("chain full", w, d, c);
        run<4, 1, 0, 1>("skew full", w, d, c);
    }
    return 0;
}
