// ubench_copy.hip -- achievable HBM rate for the one-generation kernel's traffic shape on gfx950:
// a 512 MiB -> 512 MiB copy in 8 KiB rows (65536-cell packed rows), each wave streaming a column
// chunk of 1 KiB (16 B per lane) down a band of rows, grids of W waves per CU, with or without
// non-temporal stores, P loads in flight per wave.  Prints GB/s of read + write bytes.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kRowWords = 2048, kRows = 65536;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int P, int NT>
__global__ __launch_bounds__(256) void copy_rows(const v4u *__restrict__ in, v4u *__restrict__ out,
                                                 int band) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int chunk = wave % 8, b = wave / 8;
    const int y0 = b * band;
    const int64_t col = chunk * 64 + lane;  // in v4u units; row = 512 v4u
    v4u buf[P];
#pragma unroll
    for (int u = 0; u < P; ++u) buf[u] = in[(int64_t)(y0 + u) * 512 + col];
    for (int y = 0; y < band; y += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            v4u v = buf[u];
            const int yn = y + u + P < band ? y + u + P : band - 1;
            buf[u] = in[(int64_t)(y0 + yn) * 512 + col];
            v4u *dst = out + (int64_t)(y0 + y + u) * 512 + col;
            if (NT) __builtin_nontemporal_store(v, dst);
            else *dst = v;
        }
    }
}

// Linear grid-stride float4 copy (the classic streaming copy) for comparison.
template <int NT>
__global__ __launch_bounds__(256) void copy_linear(const v4u *__restrict__ in, v4u *__restrict__ out,
                                                   int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        v4u v = in[i];
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}
template <int NT, int U>
__global__ __launch_bounds__(256) void copy_linear_u(const v4u *__restrict__ in, v4u *__restrict__ out,
                                                     int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = in[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], out + i + u * stride);
            else out[i + u * stride] = v[u];
        }
    }
}
template <class F>
void time_it(const char *name, F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    (void)hipEventRecord(a);
    const int it = 50;
    for (int i = 0; i < it; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double t = ms / 1e3 / it;
    printf("%s: %.1f us  %.0f GB/s\n", name, t * 1e6, 2.0 * kRows * kRowWords * 4 / t / 1e9);
}

template <int P, int NT>
void run(const v4u *in, v4u *out, int wpc, int cus) {
    const int waves = wpc * cus;
    const int band = kRows / (waves / 8);
    const int blocks = waves / 4;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((copy_rows<P, NT>), dim3(blocks), dim3(256), 0, 0, in, out, band);
    hipEventRecord(a);
    const int it = 50;
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL((copy_rows<P, NT>), dim3(blocks), dim3(256), 0, 0, in, out, band);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double t = ms / 1e3 / it;
    printf("P=%d NT=%d waves/CU=%d band=%d: %.1f us  %.0f GB/s\n", P, NT, wpc, band, t * 1e6,
           2.0 * kRows * kRowWords * 4 / t / 1e9);
}

int main() {
    const size_t bytes = (size_t)kRows * kRowWords * 4;
    v4u *in, *out;
    hipMalloc(&in, bytes);
    hipMalloc(&out, bytes);
    hipMemset(in, 0x5a, bytes);
    int cus = 256;
    const int64_t n = (int64_t)bytes / 16;  // n is a multiple of 256 * 4 * blocks below
    for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
        char nm[96];
        snprintf(nm, sizeof nm, "linear blocks=%d NT=0", blocks);
        time_it(nm, [&] { hipLaunchKernelGGL((copy_linear<0>), dim3(blocks), dim3(256), 0, 0, in, out, n); });
        snprintf(nm, sizeof nm, "linear blocks=%d NT=1", blocks);
        time_it(nm, [&] { hipLaunchKernelGGL((copy_linear<1>), dim3(blocks), dim3(256), 0, 0, in, out, n); });
        snprintf(nm, sizeof nm, "linear4 blocks=%d NT=1", blocks);
        time_it(nm, [&] { hipLaunchKernelGGL((copy_linear_u<1, 4>), dim3(blocks), dim3(256), 0, 0, in, out, n); });
    }
    for (int wpc : {4, 8, 16, 32}) {
        run<4, 0>(in, out, wpc, cus);
        run<4, 1>(in, out, wpc, cus);
        run<8, 1>(in, out, wpc, cus);
        run<2, 1>(in, out, wpc, cus);
    }
    return 0;
}
