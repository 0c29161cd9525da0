// golhip_kernels.hip -- the supporting gfx950 kernels of libgolhip (counts finalize, PGM pack /
// unpack, random init, popcount, alive-cell / flip extraction, word I/O) and the dispatchers of
// the hot-path stencil, whose kernels live in golhip_stencil.hpp (one TU per launch depth:
// stencil_k*.hip, stencil_split.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "golhip_internal.hpp"

namespace golhip {
namespace {


// Per-generation counts of a launch whose slots were not finalized in-kernel: block j sums
// generation j's kCountSlots slots (one per lane) and re-zeroes them.
__global__ void count_finalize(unsigned long long *slots, unsigned long long *counts) {
    const int j = blockIdx.x, lane = threadIdx.x;
    unsigned long long *sl = &slots[j * kCountSlots + lane];
    unsigned long long x = *sl;
    *sl = 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if (lane == 0) counts[j] = x;
}

// ------------------------------------------------------------------ board I/O (gol/io.go)
__global__ void pack_rows(const uint8_t *__restrict__ bytes, int64_t rows, int64_t width,
                          int32_t wd, uint32_t *__restrict__ row0, int64_t pitch) {
    const int64_t n = rows * wd;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / wd;
        const int32_t col = (int32_t)(i - y * wd);
        const uint8_t *r = bytes + y * width;
        uint32_t v = 0;
        if ((width & 31) == 0) {
            const int64_t x0 = ((int64_t)col * 32) % width;
            const uint4 *q = reinterpret_cast<const uint4 *>(r + x0);
            const uint4 lo = q[0], hi = q[1];
            const uint32_t w8[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    v |= (uint32_t)(((w8[k] >> (8 * b)) & 0xffu) != 0) << (4 * k + b);
        } else {
            for (int b = 0; b < 32; ++b) {
                const int64_t x = ((int64_t)col * 32 + b) % width;
                v |= (uint32_t)(r[x] != 0) << b;
            }
        }
        row0[y * pitch + col] = v;
    }
}

__global__ void unpack_rows(const uint32_t *__restrict__ row0, int64_t pitch, int64_t rows,
                            int64_t width, uint8_t *__restrict__ bytes) {
    if ((width & 15) == 0) {
        const int64_t per_row = width / 16, n = rows * per_row;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
             i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t y = i / per_row, t = i - y * per_row, x0 = t * 16;
            const uint32_t bits = (row0[y * pitch + (x0 >> 5)] >> (x0 & 31)) & 0xffffu;
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t w = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) w |= (((bits >> (4 * k + b)) & 1u) * 0xffu) << (8 * b);
                o[k] = w;
            }
            *reinterpret_cast<uint4 *>(bytes + y * width + x0) = make_uint4(o[0], o[1], o[2], o[3]);
        }
    } else {
        const int64_t n = rows * width;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
             i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t y = i / width, x = i - y * width;
            bytes[i] = ((row0[y * pitch + (x >> 5)] >> (x & 31)) & 1u) ? 255 : 0;
        }
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ void init_random_rows(uint32_t *__restrict__ row0, int64_t pitch, int64_t rows,
                                 int64_t gy0, int64_t width, int32_t wd, uint64_t seed,
                                 uint32_t density) {
    const uint64_t g = 0x9E3779B97F4A7C15ULL;
    const int64_t n = rows * wd, wpr = width / 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / wd;
        const int32_t col = (int32_t)(i - y * wd);
        const int64_t gy = gy0 + y;
        const int64_t x0 = ((int64_t)col * 32) % width;
        uint32_t v = 0;
        if (density == 0x80000000u) {
            const uint64_t wi = (uint64_t)gy * wpr + (uint64_t)(x0 >> 6);
            const uint64_t w = splitmix64(seed + (wi + 1) * g);
            v = (x0 & 32) ? (uint32_t)(w >> 32) : (uint32_t)w;
        } else {
            for (int b = 0; b < 32; ++b) {
                const uint64_t c = (uint64_t)gy * width + (uint64_t)(x0 + b);
                const uint32_t d = (uint32_t)splitmix64(seed + (c + 1) * g);
                v |= (uint32_t)(d < density) << b;
            }
        }
        row0[y * pitch + col] = v;
    }
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Alive cells of rows x wd words (wd % 4 == 0: the torus width is a multiple of 128): a block
// per row at a time, 16-byte loads, no per-element index division.
__global__ void popcount_rows(const uint32_t *__restrict__ row0, int64_t pitch, int64_t rows,
                              int32_t wd, unsigned long long *__restrict__ out) {
    __shared__ unsigned long long part[4];
    const int q = wd / 4;
    unsigned long long c = 0;
    for (int64_t y = blockIdx.x; y < rows; y += gridDim.x) {
        const uint4 *r = reinterpret_cast<const uint4 *>(row0 + y * pitch);
        for (int i = threadIdx.x; i < q; i += blockDim.x) {
            const uint4 v = r[i];
            c += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) +
                 __builtin_popcount(v.w);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
        if (t) atomicAdd(out, t);
    }
}

// ------------------------------------------------ alive-cell / flip extraction (row-major)
__device__ __forceinline__ uint32_t cell_word(const uint32_t *a, const uint32_t *b,
                                              int64_t off, int32_t col, int32_t nw,
                                              uint32_t lastmask) {
    uint32_t v = a[off];
    if (b) v ^= b[off];
    if (col == nw - 1) v &= lastmask;
    return v;
}

// Phase 1: block b counts rows [b * per, (b + 1) * per) (one wave per row at a time) into
// row_counts and their total into block_sums[b].
__global__ void extract_count(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                              int64_t pitch, int64_t rows, int64_t per, int32_t nw,
                              uint32_t lastmask, uint32_t *__restrict__ row_counts,
                              unsigned long long *__restrict__ block_sums) {
    __shared__ unsigned long long part[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t y0 = (int64_t)blockIdx.x * per, y1 = min(rows, y0 + per);
    unsigned long long tot = 0;
    for (int64_t y = y0 + wv; y < y1; y += 4) {
        uint32_t c = 0;
        for (int32_t col = lane; col < nw; col += 64)
            c += __builtin_popcount(cell_word(a, b, y * pitch + col, col, nw, lastmask));
        c = wave_sum_u32(c);
        if (lane == 0) row_counts[y] = c;
        tot += c;
    }
    if (lane == 0) part[wv] = tot;
    __syncthreads();
    if (threadIdx.x == 0) block_sums[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// Inclusive scan of one value per thread over a 256-thread block (4 waves, shuffles + LDS).
__device__ __forceinline__ unsigned long long block_scan_incl(unsigned long long v,
                                                               unsigned long long *wsum) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    unsigned long long add = 0;
    for (int w = 0; w < wv; ++w) add += wsum[w];
    __syncthreads();
    return v + add;
}

// Phase 2 (one block of kScanBlocks threads): block_sums -> their exclusive scan, in place;
// offsets[rows] = the total.
__global__ void extract_scan_blocks(unsigned long long *__restrict__ block_sums, int nb,
                                    unsigned long long *__restrict__ total) {
    __shared__ unsigned long long wsum[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    unsigned long long v = t < nb ? block_sums[t] : 0ull, x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long u = __shfl_up(x, off, 64);
        if (lane >= off) x += u;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    unsigned long long add = 0;
    for (int w = 0; w < wv; ++w) add += wsum[w];
    if (t < nb) block_sums[t] = add + x - v;
    if (t == (int)blockDim.x - 1) *total = add + x;
}

// Phase 3: block b writes the exclusive offsets of its rows (tiles of 256 rows, block scans).
__global__ void extract_scan_rows(const uint32_t *__restrict__ row_counts, int64_t rows, int64_t per,
                                  const unsigned long long *__restrict__ block_offs,
                                  unsigned long long *__restrict__ offsets) {
    __shared__ unsigned long long wsum[4];
    __shared__ unsigned long long carry;
    const int64_t y0 = (int64_t)blockIdx.x * per, y1 = min(rows, y0 + per);
    unsigned long long run = block_offs[blockIdx.x];
    for (int64_t t0 = y0; t0 < y1; t0 += 256) {
        const int64_t y = t0 + threadIdx.x;
        const unsigned long long v = y < y1 ? row_counts[y] : 0ull;
        const unsigned long long incl = block_scan_incl(v, wsum);
        if (y < y1) offsets[y] = run + incl - v;
        if (threadIdx.x == 255) carry = incl;
        __syncthreads();
        run += carry;
        __syncthreads();
    }
}

// Cells of slot t = rows [t * slot_rows, (t+1) * slot_rows) of a tall board: counts[t].
__global__ void extract_slot_counts(const unsigned long long *__restrict__ offsets,
                                    int64_t slot_rows, int64_t slots,
                                    unsigned long long *__restrict__ counts) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < slots;
         t += (int64_t)gridDim.x * blockDim.x)
        counts[t] = offsets[(t + 1) * slot_rows] - offsets[t * slot_rows];
}

// (x, y) of every cell, row-major; a tall board of slots reports y within its slot
// (y = gy0 + row % slot_rows), slot-major.  X16: x only, as uint16 (width <= 65536; the row of
// entry i is given by the offsets table, golhip_step_flips_rows) -- a quarter of the bytes.
template <bool X16>
__global__ void extract_emit(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                             int64_t pitch, int64_t rows, int32_t nw, uint32_t lastmask,
                             const unsigned long long *__restrict__ offsets, int64_t gy0,
                             int64_t slot_rows, int32_t *__restrict__ xy, uint64_t cap) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t y = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); y < rows;
         y += nwaves) {
        unsigned long long base = offsets[y];
        if (base >= cap) continue;
        for (int32_t c0 = 0; c0 < nw; c0 += 64) {
            const int32_t col = c0 + lane;
            uint32_t v = col < nw ? cell_word(a, b, y * pitch + col, col, nw, lastmask) : 0u;
            const uint32_t cnt = __builtin_popcount(v);
            uint32_t incl = cnt;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            unsigned long long pos = base + (incl - cnt);
            while (v) {
                const int bit = __builtin_ctz(v);
                v &= v - 1;
                if (pos < cap) {
                    if constexpr (X16) {
                        reinterpret_cast<uint16_t *>(xy)[pos] = (uint16_t)(col * 32 + bit);
                    } else {
                        xy[2 * pos] = col * 32 + bit;
                        xy[2 * pos + 1] = (int32_t)(gy0 + y % slot_rows);
                    }
                }
                ++pos;
            }
            base += __shfl(incl, 63, 64);
        }
    }
}

__global__ void words_out(const uint32_t *__restrict__ row0, int64_t pitch, int64_t rows,
                          int64_t wpr, uint64_t *__restrict__ words) {
    const int64_t n = rows * wpr;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / wpr, j = i - y * wpr;
        const uint32_t *r = row0 + y * pitch + 2 * j;
        words[i] = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
    }
}

__global__ void words_in(const uint64_t *__restrict__ words, int64_t rows, int64_t wpr,
                         int32_t wd, uint32_t *__restrict__ row0, int64_t pitch) {
    const int64_t n = rows * wd;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / wd;
        const int32_t col = (int32_t)(i - y * wd);
        const int64_t lw = ((int64_t)col / 2) % wpr;  // logical word (torus replication)
        const uint64_t w = words[y * wpr + lw];
        row0[y * pitch + col] = (col & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
    }
}
inline unsigned grid_for(int64_t n, int threads = 256, int64_t cap = 8192) {
    int64_t g = (n + threads - 1) / threads;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace

KernelExtras &kernel_extras() {
    static KernelExtras x;  // filled by the tuning library's TUs; empty in production
    return x;
}

static bool prod_depth(int K) {
    switch (K) {
#define GOLHIP_X(KK) case KK:
        GOLHIP_STENCIL_DEPTHS(GOLHIP_X)
#undef GOLHIP_X
        return true;
        default: return false;
    }
}

bool stencil_k_supported(int K) {
    return prod_depth(K) || (K >= 1 && K <= kMaxK && kernel_extras().stencil[K] != nullptr);
}

// The per-depth production launchers live in stencil_k<K>.hip (one TU per depth); any other
// variant or depth is a kernel_extras() entry (the tuning library), or not in this library.
hipError_t launch_stencil(int K, int variant, const uint32_t *in_row0, uint32_t *out_row0,
                          const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    if (variant == kVariantProd) {
        switch (K) {
#define GOLHIP_X(KK) \
    case KK: return launch_stencil_k##KK(in_row0, out_row0, p, slots, s);
            GOLHIP_STENCIL_DEPTHS(GOLHIP_X)
#undef GOLHIP_X
            default: break;
        }
    }
    if (K >= 1 && K <= kMaxK && kernel_extras().stencil[K])
        return kernel_extras().stencil[K](variant, in_row0, out_row0, p, slots, s);
    return hipErrorInvalidValue;
}

hipError_t warm_stencils(int variant, hipStream_t s) {
    hipError_t e = hipSuccess;
    const KernelExtras &x = kernel_extras();
    for (int K = 1; K <= kMaxK && e == hipSuccess; ++K) {
        if (variant != kVariantProd || !prod_depth(K)) {
            if (x.stencil_warm[K]) e = x.stencil_warm[K](variant, s);
            continue;
        }
        switch (K) {
#define GOLHIP_X(KK) \
    case KK: e = warm_stencil_k##KK(s); break;
            GOLHIP_STENCIL_DEPTHS(GOLHIP_X)
#undef GOLHIP_X
            default: break;
        }
    }
    if (e == hipSuccess && x.split_warm) e = x.split_warm(s);
    if (e == hipSuccess) e = warm_stencil_tile(s);
    return e;
}

int stencil_waves_per_cu(int K, int variant) {
    const void *fn = nullptr;
    if (variant == kVariantProd) {
        switch (K) {
#define GOLHIP_X(KK) \
    case KK: fn = stencil_fn_k##KK(); break;
            GOLHIP_STENCIL_DEPTHS(GOLHIP_X)
#undef GOLHIP_X
            default: break;
        }
    }
    if (!fn && K >= 1 && K <= kMaxK && kernel_extras().stencil_fn[K]) fn = kernel_extras().stencil_fn[K](variant);
    if (!fn) return 4;
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, 256, lds_pad_bytes()) != hipSuccess || blocks < 1)
        return 4;
    return blocks * 4;  // 256-thread blocks = 4 waves
}

hipError_t launch_count_finalize(int K, unsigned long long *slots, unsigned long long *counts,
                                 hipStream_t s) {
    static_assert(kCountSlots == 64, "one slot per lane");
    hipLaunchKernelGGL(count_finalize, dim3(K), dim3(64), 0, s, slots, counts);
    return hipGetLastError();
}

hipError_t launch_pack(const uint8_t *bytes, int64_t rows, int64_t width, int32_t wd,
                       uint32_t *row0, int64_t pitch, hipStream_t s) {
    hipLaunchKernelGGL(pack_rows, dim3(grid_for(rows * wd)), dim3(256), 0, s, bytes, rows, width,
                       wd, row0, pitch);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t *row0, int64_t pitch, int64_t rows, int64_t width,
                         uint8_t *bytes, hipStream_t s) {
    const int64_t n = (width & 15) == 0 ? rows * (width / 16) : rows * width;
    hipLaunchKernelGGL(unpack_rows, dim3(grid_for(n)), dim3(256), 0, s, row0, pitch, rows, width,
                       bytes);
    return hipGetLastError();
}

hipError_t launch_init_random(uint32_t *row0, int64_t pitch, int64_t rows, int64_t gy0,
                              int64_t width, int32_t wd, uint64_t seed, uint32_t density_q32,
                              hipStream_t s) {
    hipLaunchKernelGGL(init_random_rows, dim3(grid_for(rows * wd)), dim3(256), 0, s, row0, pitch,
                       rows, gy0, width, wd, seed, density_q32);
    return hipGetLastError();
}

hipError_t launch_popcount(const uint32_t *row0, int64_t pitch, int64_t rows, int32_t wd,
                           unsigned long long *out, hipStream_t s) {
    const unsigned blocks = (unsigned)std::min<int64_t>(std::max<int64_t>(rows, 1), 4096);
    hipLaunchKernelGGL(popcount_rows, dim3(blocks), dim3(256), 0, s, row0, pitch, rows, wd, out);
    return hipGetLastError();
}

static void extract_geometry(int64_t width, int32_t &nw, uint32_t &lastmask) {
    nw = (int32_t)((width + 31) / 32);
    lastmask = (width & 31) ? ((1u << (width & 31)) - 1u) : 0xffffffffu;
}

hipError_t launch_extract_count(const uint32_t *a, const uint32_t *b, int64_t pitch,
                                int64_t rows, int64_t width, uint32_t *row_counts,
                                unsigned long long *offsets, unsigned long long *block_sums,
                                hipStream_t s) {
    int32_t nw;
    uint32_t lastmask;
    extract_geometry(width, nw, lastmask);
    // contiguous row ranges of >= 16 rows per block, at most kScanBlocks blocks
    const int64_t per = std::max<int64_t>(16, (rows + kScanBlocks - 1) / kScanBlocks);
    const int nb = (int)std::max<int64_t>(1, (rows + per - 1) / per);
    hipLaunchKernelGGL(extract_count, dim3(nb), dim3(256), 0, s, a, b, pitch, rows, per, nw,
                       lastmask, row_counts, block_sums);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(extract_scan_blocks, dim3(1), dim3(kScanBlocks), 0, s, block_sums, nb,
                       offsets + rows);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(extract_scan_rows, dim3(nb), dim3(256), 0, s, row_counts, rows, per,
                       block_sums, offsets);
    return hipGetLastError();
}

hipError_t launch_extract_emit(const uint32_t *a, const uint32_t *b, int64_t pitch,
                               int64_t rows, int64_t width, const unsigned long long *offsets,
                               int64_t gy0, int64_t slot_rows, int32_t *xy, uint64_t cap,
                               hipStream_t s) {
    int32_t nw;
    uint32_t lastmask;
    extract_geometry(width, nw, lastmask);
    const unsigned blocks = grid_for(rows * 64, 256, 16384);
    hipLaunchKernelGGL(extract_emit<false>, dim3(blocks), dim3(256), 0, s, a, b, pitch, rows, nw,
                       lastmask, offsets, gy0, slot_rows, xy, cap);
    return hipGetLastError();
}

hipError_t launch_extract_emit_x16(const uint32_t *a, const uint32_t *b, int64_t pitch,
                                   int64_t rows, int64_t width, const unsigned long long *offsets,
                                   uint16_t *x, uint64_t cap, hipStream_t s) {
    int32_t nw;
    uint32_t lastmask;
    extract_geometry(width, nw, lastmask);
    const unsigned blocks = grid_for(rows * 64, 256, 16384);
    hipLaunchKernelGGL(extract_emit<true>, dim3(blocks), dim3(256), 0, s, a, b, pitch, rows, nw,
                       lastmask, offsets, (int64_t)0, rows, reinterpret_cast<int32_t *>(x), cap);
    return hipGetLastError();
}

hipError_t launch_extract_slot_counts(const unsigned long long *offsets, int64_t slot_rows,
                                      int64_t slots, unsigned long long *counts, hipStream_t s) {
    hipLaunchKernelGGL(extract_slot_counts, dim3(grid_for(slots, 256, 64)), dim3(256), 0, s,
                       offsets, slot_rows, slots, counts);
    return hipGetLastError();
}

hipError_t launch_words_out(const uint32_t *row0, int64_t pitch, int64_t rows, int64_t width,
                            uint64_t *words, hipStream_t s) {
    const int64_t wpr = width / 64;
    hipLaunchKernelGGL(words_out, dim3(grid_for(rows * wpr)), dim3(256), 0, s, row0, pitch, rows,
                       wpr, words);
    return hipGetLastError();
}

hipError_t launch_words_in(const uint64_t *words, int64_t rows, int64_t width, int32_t wd,
                           uint32_t *row0, int64_t pitch, hipStream_t s) {
    const int64_t wpr = width / 64;
    hipLaunchKernelGGL(words_in, dim3(grid_for(rows * wd)), dim3(256), 0, s, words, rows, wpr, wd,
                       row0, pitch);
    return hipGetLastError();
}

}  // namespace golhip