// fetch_cal.hip -- calibration of rocprofv3's FETCH_SIZE for the access patterns this library's
// kernels use (MI355X_MICROARCH.md: FETCH_SIZE counts exactly 1/2 of a 16-B-per-lane contiguous
// streaming read on gfx950; other widths are uncalibrated).  Each kernel reads every byte of a
// 2 GiB buffer exactly once (far past the 256 MiB Infinity Cache), so bytes / (FETCH_SIZE x 1024)
// is the correction factor of that pattern:
//   k_contig16  lane t of a wave reads 16 B at 16 t (+ 1 KiB per step): the calibrated pattern
//   k_piece16   lane t reads 4 x 16 B at 64 t (+ 16 j): pw_load_piece since round 4 (a K-thread
//               workgroup, thread t owns limbs [8 t, 8 t + 8) of a 2048-limb coefficient)
//   k_piece8    lane t reads 8 x 8 B at 64 t (+ 8 j): pw_load_piece before round 4
// Run: rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -- ./fetch_cal
// build: hipcc --offload-arch=gfx950 -O3 -o fetch_cal fetch_cal.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint64_t u64;
typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// one workgroup of 256 threads per 16 KiB coefficient (2048 limbs), like k_pwss<18, 8, *>
__global__ __launch_bounds__(256) void k_contig16(const u64 *src, u64 *sink)
{
    const u64 *c = src + (size_t)blockIdx.x * 2048;
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const v2u v = *(const v2u *)(c + 2 * (threadIdx.x + 256 * j));
        acc += v.x ^ v.y;
    }
    if (acc == 0x123456789abcdefull) sink[0] = acc;   // keeps the loads
}

__global__ __launch_bounds__(256) void k_piece16(const u64 *src, u64 *sink)
{
    const u64 *c = src + (size_t)blockIdx.x * 2048 + 8 * threadIdx.x;
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const v2u v = *(const v2u *)(c + j);
        acc += v.x ^ v.y;
    }
    if (acc == 0x123456789abcdefull) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_piece8(const u64 *src, u64 *sink)
{
    const u64 *c = src + (size_t)blockIdx.x * 2048 + 8 * threadIdx.x;
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += c[j];
    if (acc == 0x123456789abcdefull) sink[0] = acc;
}

int main()
{
    const size_t bytes = (size_t)2 << 30, coefs = bytes / (2048 * 8);
    u64 *src, *sink;
    CHK(hipMalloc(&src, bytes));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(src, 1, bytes));
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_contig16, dim3((unsigned)coefs), dim3(256), 0, 0, src, sink);
    hipLaunchKernelGGL(k_piece16, dim3((unsigned)coefs), dim3(256), 0, 0, src, sink);
    hipLaunchKernelGGL(k_piece8, dim3((unsigned)coefs), dim3(256), 0, 0, src, sink);
    CHK(hipDeviceSynchronize());
    printf("each kernel read %zu bytes once\n", bytes);
    return 0;
}
