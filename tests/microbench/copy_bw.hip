// copy_bw.hip -- what one pass over C1-sized coefficient arrays can cost: a wave
// copies K coefficients of L limbs (8 B per lane per row, or 16 B per lane per row).
// build: hipcc --offload-arch=gfx950 -O3 -o copy_bw copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint64_t u64;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int K, int W>   // W = 8 or 16 bytes per lane per access
__global__ __launch_bounds__(256) void k_copy(const u64 *src, u64 *dst, int l, long ncoef)
{
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave * K >= ncoef) return;
    if (W == 8) {
        u64 v[K][8];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int m = 64 * u + lane;
                v[k][u] = m < l ? src[(wave * K + k) * l + m] : 0;
            }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int m = 64 * u + lane;
                if (m < l) dst[(wave * K + k) * l + m] = v[k][u] + 1;
            }
    } else {
        typedef unsigned long long v2 __attribute__((ext_vector_type(2)));
        v2 v[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = 128 * u + 2 * lane;
                v[k][u] = m < l ? *(const v2 *)(src + (wave * K + k) * l + m) : v2{0, 0};
            }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = 128 * u + 2 * lane;
                if (m < l) *(v2 *)(dst + (wave * K + k) * l + m) = v[k][u] + 1;
            }
    }
}

template <int K, int W>
static int run(const char *name, u64 *a, u64 *b, int l, long ncoef, int reps)
{
    const long waves = (ncoef + K - 1) / K;
    dim3 grid((unsigned)((waves * 64 + 255) / 256));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy<K, W>), grid, dim3(256), 0, 0, a, b, l, ncoef);
    CHK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_copy<K, W>), grid, dim3(256), 0, 0, (i & 1) ? b : a, (i & 1) ? a : b, l, ncoef);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / reps, bytes = 2.0 * ncoef * l * 8;
    printf("%-10s l=%d ncoef=%ld K=%d W=%d: %8.2f us/launch  %7.1f GB/s\n", name, l, ncoef, K, W, us, bytes / us * 1e-3);
    return 0;
}

int main()
{
    const int l = 256;
    for (long ncoef : {8192L, 65536L, 524288L}) {
        u64 *a, *b;
        CHK(hipMalloc(&a, ncoef * l * 8));
        CHK(hipMalloc(&b, ncoef * l * 8));
        CHK(hipMemset(a, 1, ncoef * l * 8));
        const int reps = ncoef > 100000 ? 20 : 200;
        run<1, 8>("copy", a, b, l, ncoef, reps);
        run<2, 8>("copy", a, b, l, ncoef, reps);
        run<8, 8>("copy", a, b, l, ncoef, reps);
        run<1, 16>("copy", a, b, l, ncoef, reps);
        run<2, 16>("copy", a, b, l, ncoef, reps);
        run<8, 16>("copy", a, b, l, ncoef, reps);
        CHK(hipFree(a));
        CHK(hipFree(b));
    }
    return 0;
}
