// Microbenchmark: 32x32->64 multiply-accumulate throughput on gfx950 (VALU, wave64).
// Variants: (a) v_mad_u64_u32 acc-chain + v_addc (inline asm), (b) compiler u64 MAC,
// (c) v_mul_lo_u32 + v_mul_hi_u32.  Each thread runs independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint64_t u64; typedef uint32_t u32;

#define CH 8
__global__ __launch_bounds__(256) void k_asm(const u32 *in, u64 *out, int iters) {
    u32 a[CH], b = in[threadIdx.x] | 1; u64 acc[CH]; u32 h[CH];
    for (int c = 0; c < CH; ++c) { a[c] = in[threadIdx.x + c + 1]; acc[c] = c; h[c] = 0; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            u64 cy;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_addc_co_u32_e64 %4, %1, 0, %4, %1"
                         : "+v"(acc[c]), "=&s"(cy) : "v"(a[c]), "v"(b), "v"(h[c]) );
            (void)cy;
        }
        b += 0x9e37;
    }
    u64 s = 0; for (int c = 0; c < CH; ++c) s += acc[c] + h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mad(const u32 *in, u64 *out, int iters) {
    u32 a[CH], b = in[threadIdx.x] | 1; u64 acc[CH];
    for (int c = 0; c < CH; ++c) { a[c] = in[threadIdx.x + c + 1]; acc[c] = c; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            u64 cy;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=&s"(cy) : "v"(a[c]), "v"(b));
            (void)cy;
        }
        b += 0x9e37;
    }
    u64 s = 0; for (int c = 0; c < CH; ++c) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cc(const u32 *in, u64 *out, int iters) {
    u32 a[CH], b = in[threadIdx.x] | 1; u64 acc[CH]; u32 h[CH];
    for (int c = 0; c < CH; ++c) { a[c] = in[threadIdx.x + c + 1]; acc[c] = c; h[c] = 0; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) { u64 p = (u64)a[c] * b; acc[c] += p; h[c] += acc[c] < p; }
        b += 0x9e37;
    }
    u64 s = 0; for (int c = 0; c < CH; ++c) s += acc[c] + h[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mulhl(const u32 *in, u64 *out, int iters) {
    u32 a[CH], b = in[threadIdx.x] | 1; u32 lo[CH], hi[CH];
    for (int c = 0; c < CH; ++c) { a[c] = in[threadIdx.x + c + 1]; lo[c] = c; hi[c] = 0; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) { lo[c] += a[c] * b; hi[c] += __umulhi(a[c], b); }
        b += 0x9e37;
    }
    u64 s = 0; for (int c = 0; c < CH; ++c) s += lo[c] + hi[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_add(const u32 *in, u64 *out, int iters) {
    u32 a[CH], b = in[threadIdx.x] | 1; u32 lo[CH];
    for (int c = 0; c < CH; ++c) { a[c] = in[threadIdx.x + c + 1]; lo[c] = c; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) { lo[c] = lo[c] + (a[c] ^ b); }
        b += 0x9e37;
    }
    u64 s = 0; for (int c = 0; c < CH; ++c) s += lo[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    u32 *in; u64 *out;
    hipMalloc(&in, 4096 * 4); hipMalloc(&out, (size_t)blocks * threads * 8);
    hipMemset(in, 0x5b, 4096 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    struct { const char *name; void (*k)(const u32*, u64*, int); double ops_per_iter; } ks[] = {
        {"asm v_mad_u64_u32+v_addc (MAC)", k_asm, CH}, {"asm v_mad_u64_u32 alone", k_mad, CH}, {"compiler u64 MAC", k_cc, CH},
        {"v_mul_lo+v_mul_hi (MAC halves)", k_mulhl, CH}, {"v_add_u32+xor (2 simple ops)", k_add, CH}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            double n = (double)blocks * threads * iters * k.ops_per_iter;
            if (rep) printf("%-36s %8.3f ms  %8.2f T/s (per lane-op unit)\n", k.name, ms, n / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
