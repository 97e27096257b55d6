// pass_bw.hip -- the HBM ceiling of a k_rpass-shaped pass: how fast can one in-place pass over
// C3's coefficient arrays (2 x 39680 x 2048 limbs = 1.3 GB, read + written) go when a
// workgroup holds a whole butterfly group in registers (G coefficients x 16 KB), compared
// with a plain streaming copy of the same bytes.  No arithmetic: memory structure only.
// build: hipcc --offload-arch=gfx950 -O3 -o pass_bw pass_bw.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint64_t u64;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// grid-stride in-place streaming: every thread 4 x 16 B in flight
__global__ __launch_bounds__(256) void k_stream(v4u *x, long n16)
{
    const long nt = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += 4 * nt) {
        v4u v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i + k * nt < n16 ? x[i + k * nt] : v4u{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k * nt < n16) x[i + k * nt] = v[k] + 1u;
    }
}

// out-of-place streaming (ping-pong passes): read x, write y
__global__ __launch_bounds__(256) void k_stream_oop(const v4u *x, v4u *y, long n16)
{
    const long nt = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += 4 * nt) {
        v4u v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i + k * nt < n16 ? x[i + k * nt] : v4u{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k * nt < n16) y[i + k * nt] = v[k] + 1u;
    }
}

// one workgroup = one group of G coefficients of L limbs at stride S coefficients (a column
// pass: positions pos0 + i * S); NT threads, each 16 B x (L / 2 / NT) per coefficient.
// LDS: `lds` bytes of dummy allocation (k_rpass: 74 KB at l = 2048, G = 8 -> 2 WGs per CU).
template <int G, int NT, int L>
__global__ __launch_bounds__(NT) void k_group(v4u *x, int stride, int ngroups_per_col, int spin, v4u *y = nullptr,
                                              int stagger = 0, int unit = 0)
{
    extern __shared__ unsigned char smem[];
    // stagger (round 5): the first workgroup on each CU waits (b mod stagger) units of ~3.4 us
    // before its loads, so CUs that would otherwise load and compute in lockstep (identical
    // groups started together) are spread over the period: while some compute, others load
    if (stagger && blockIdx.x < 256) {
        const int n = (int)(blockIdx.x % stagger) * unit;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }
    constexpr int R = L / 2 / NT;
    const int col = blockIdx.x / ngroups_per_col, grp = blockIdx.x % ngroups_per_col;
    const int t = threadIdx.x;
    v4u v[G][R];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const long slot = (long)(grp + i * ngroups_per_col) * stride + col;
#pragma unroll
        for (int r = 0; r < R; ++r) v[i][r] = x[slot * (L / 2) + t + NT * r];
    }
    __syncthreads();
    if (spin) {   // a stand-in for the levels: VALU work on the registers
        for (int s = 0; s < spin; ++s)
#pragma unroll
            for (int i = 0; i < G; ++i)
#pragma unroll
                for (int r = 0; r < R; ++r) v[i][r] = v[i][r] * 3u + (unsigned)s;
        if (t == 0) smem[0] = (unsigned char)v[0][0].x;
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const long slot = (long)(grp + i * ngroups_per_col) * stride + col;
#pragma unroll
        for (int r = 0; r < R; ++r) (y ? y : x)[slot * (L / 2) + t + NT * r] = v[i][r] + 1u;
    }
}

int main()
{
    const long NCOL = 128, NPOS = 512, L = 2048, slots = 2 * NCOL * NPOS;   // both operands: 2 x 128 columns
    const size_t bytes = (size_t)slots * L * 8;
    v4u *x;
    CHK(hipMalloc(&x, bytes));
    CHK(hipMemset(x, 1, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto report = [&](const char *name, float ms, int reps) {
        const double s = ms * 1e-3 / reps;
        printf("%-44s %8.3f ms  %6.2f TB/s (read + write of %.2f GB)\n", name, s * 1e3, 2.0 * bytes / s * 1e-12,
               bytes * 1e-9);
    };
    const int reps = 10;
    {
        const long n16 = bytes / 16;
        for (int grid : {1024, 2048, 4096, 8192}) {
            hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, x, n16);
            CHK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, x, n16);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            char nm[64];
            snprintf(nm, sizeof nm, "stream in place, grid %d x 256", grid);
            report(nm, ms, reps);
        }
    }
    // column-pass shape: 2 * 128 columns (stride 256 slots), 512 positions, G = 8 -> 64 groups per column
    const int G = 8, gpc = (int)(NPOS / G), ncols = (int)(2 * NCOL);
    for (int lds : {0, 74 * 1024, 148 * 1024}) {
        for (int spin : {0, 64, 256}) {
            auto f = k_group<8, 512, 2048>;
            if (lds > 64 * 1024) CHK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
            hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(512), lds, 0, x, ncols, gpc, spin, (v4u *)nullptr, 0, 0);
            CHK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(512), lds, 0, x, ncols, gpc, spin, (v4u *)nullptr, 0, 0);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            char nm[96];
            snprintf(nm, sizeof nm, "group G=8 NT=512 lds=%dK spin=%d", lds / 1024, spin);
            report(nm, ms, reps);
        }
    }
    for (int spin : {0, 64, 256}) {
        auto f = k_group<8, 1024, 2048>;
        const int lds = 74 * 1024;
        CHK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(1024), lds, 0, x, ncols, gpc, spin, (v4u *)nullptr, 0, 0);
        CHK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(1024), lds, 0, x, ncols, gpc, spin, (v4u *)nullptr, 0, 0);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        char nm[96];
        snprintf(nm, sizeof nm, "group G=8 NT=1024 lds=74K spin=%d", spin);
        report(nm, ms, reps);
    }
    // out of place (round 5): the same shapes reading x and writing a second
    // array y, i.e. column passes ping-ponging between two halves of a doubled array
    v4u *y;
    CHK(hipMalloc(&y, bytes));
    CHK(hipMemset(y, 2, bytes));
    {
        const long n16 = bytes / 16;
        for (int grid : {1024, 2048, 4096}) {
            hipLaunchKernelGGL(k_stream_oop, dim3(grid), dim3(256), 0, 0, x, y, n16);
            CHK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_stream_oop, dim3(grid), dim3(256), 0, 0, x, y, n16);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            char nm[64];
            snprintf(nm, sizeof nm, "stream out of place, grid %d x 256", grid);
            report(nm, ms, reps);
        }
    }
    for (int oop : {0, 1}) {
        for (int spin : {0, 16, 64}) {   // the four-level pass's shape: G = 16, NT = 1024, 148 KB LDS, one WG per CU
            auto f = k_group<16, 1024, 2048>;
            const int lds = 148 * 1024, gpc16 = (int)(NPOS / 16);
            CHK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
            hipLaunchKernelGGL(f, dim3(ncols * gpc16), dim3(1024), lds, 0, x, ncols, gpc16, spin, oop ? y : nullptr, 0, 0);
            CHK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i)
                hipLaunchKernelGGL(f, dim3(ncols * gpc16), dim3(1024), lds, 0, x, ncols, gpc16, spin, oop ? y : nullptr, 0, 0);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            char nm[96];
            snprintf(nm, sizeof nm, "group G=16 NT=1024 lds=148K spin=%d %s", spin, oop ? "out of place" : "in place");
            report(nm, ms, reps);
        }
        for (int spin : {0, 64}) {   // the three-level pass's shape out of place
            auto f = k_group<8, 512, 2048>;
            const int lds = 74 * 1024;
            CHK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
            hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(512), lds, 0, x, ncols, gpc, spin, oop ? y : nullptr, 0, 0);
            CHK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i)
                hipLaunchKernelGGL(f, dim3(ncols * gpc), dim3(512), lds, 0, x, ncols, gpc, spin, oop ? y : nullptr, 0, 0);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            char nm[96];
            snprintf(nm, sizeof nm, "group G=8 NT=512 lds=74K spin=%d %s", spin, oop ? "out of place" : "in place");
            report(nm, ms, reps);
        }
    }
    // staggered starts (round 5): the four-level shape with the levels' worth of compute
    for (int spin : {16, 32, 64}) {
        for (int st : {0, 2, 4, 8}) {
            for (int unit : {1, 2, 4}) {
                if (!st && unit > 1) continue;
                auto f = k_group<16, 1024, 2048>;
                const int lds = 148 * 1024, gpc16 = (int)(NPOS / 16);
                CHK(hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
                hipLaunchKernelGGL(f, dim3(ncols * gpc16), dim3(1024), lds, 0, x, ncols, gpc16, spin, (v4u *)nullptr, st, unit);
                CHK(hipEventRecord(e0));
                for (int i = 0; i < reps; ++i)
                    hipLaunchKernelGGL(f, dim3(ncols * gpc16), dim3(1024), lds, 0, x, ncols, gpc16, spin, (v4u *)nullptr, st,
                                       unit);
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                char nm[96];
                snprintf(nm, sizeof nm, "G=16 NT=1024 148K spin=%d stagger=%d unit=%d", spin, st, unit);
                report(nm, ms, reps);
            }
        }
    }
    for (int spin : {0, 64}) {   // G = 4 (two levels per pass), 4 WGs per CU
        auto f = k_group<4, 512, 2048>;
        const int lds = 37 * 1024;
        hipLaunchKernelGGL(f, dim3(ncols * (NPOS / 4)), dim3(512), lds, 0, x, ncols, (int)(NPOS / 4), spin, (v4u *)nullptr, 0, 0);
        CHK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(f, dim3(ncols * (NPOS / 4)), dim3(512), lds, 0, x, ncols, (int)(NPOS / 4), spin, (v4u *)nullptr, 0, 0);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        char nm[96];
        snprintf(nm, sizeof nm, "group G=4 NT=512 lds=37K spin=%d", spin);
        report(nm, ms, reps);
    }
    return 0;
}
