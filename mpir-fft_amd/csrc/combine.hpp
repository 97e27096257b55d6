// combine.hpp -- FFT_combine_bits (mul_fft.c:207-267) on the GPU: limb-parallel
// shifted sums of the canonical coefficients plus a device-wide carry lookahead.
#pragma once
#include "coeff.hpp"

// --------------------------------------------------------------------------
// combine: r = sum_{k < len} c_k 2^(k bits1), c_k < 2^N canonical.
// k_comb_sum: per output limb m, the 128-bit sum of the (at most a few)
// coefficient windows covering bits [64m, 64m + 64); lo -> lo64[m], hi -> hi32[m].
// The carry chain r = lo + (hi << 64) is then resolved by a device-wide
// carry-lookahead (k_carry_blocks -> k_carry_scan -> k_carry_apply).
// --------------------------------------------------------------------------
struct CombArgs {
    const u64 *dig;      // canonical coefficients c_k (< 2^N) in the (blocked) row layout
    int l;
    u64 N, bits1;
    long len;            // number of coefficients j1 + j2 - 1
    long m0, mcount;     // output limbs [m0, m0 + mcount); the kernel also sums limb m0 - 1
    long kbase;          // first locally stored coefficient (row r0 * NC)
    const u64 *halo;     // coefficients [kbase - H, kbase) contiguous, or null
    int H;
    int NC, cbb, ccb;    // row layout: k -> p = k / NC - r0, c = k % NC,
    long cbs;            //   slot = (c >> cbb) * cbs + p * ccb + (c & (ccb - 1))
    long r0;
    u64 *lo64;           // [mcount + 1]: index i <-> limb m0 - 1 + i
    u32 *hi32;
};

__device__ __forceinline__ const u64 *coef_ptr(const CombArgs &a, long k)
{
    if (k < a.kbase) return a.halo + (size_t)(k - (a.kbase - a.H)) * a.l;
    const long p = k / a.NC - a.r0;
    const int cc = (int)(k % a.NC);
    const long slot = (long)(cc >> a.cbb) * a.cbs + p * a.ccb + (cc & (a.ccb - 1));
    return a.dig + (size_t)slot * a.l;
}

// per output limb m: the 128-bit sum of the (few) coefficient windows covering
// bits [64m, 64m + 64)  (FFT_combine_bits, mul_fft.c:207-267)
__global__ __launch_bounds__(256) void k_comb_sum(CombArgs a)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > a.mcount) return;
    const long m = a.m0 - 1 + i;
    if (m < 0) {
        a.lo64[i] = 0;
        a.hi32[i] = 0;
        return;
    }
    const u64 P = (u64)m * 64;
    long klo = (P >= a.N) ? (long)((P - a.N) / a.bits1) : 0;
    long khi = (long)((P + 63) / a.bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    u64 slo = 0;
    u32 shi = 0;
    for (long k = klo; k <= khi; ++k) {
        const u64 st = (u64)k * a.bits1;
        const u64 *cp = coef_ptr(a, k);
        u64 v;
        if (st > P) {
            v = cp[0] << (st - P);
        } else {
            const u64 o = P - st;
            const long q = (long)(o >> 6);
            const int s = (int)(o & 63);
            const u64 w0 = (q < a.l) ? cp[q] : 0;
            const u64 w1 = (s && q + 1 < a.l) ? cp[q + 1] : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
        }
        u64 t;
        shi += add_ovf(slo, v, &t);
        slo = t;
    }
    a.lo64[i] = slo;
    a.hi32[i] = shi;
}

// local limb m (0-based) of the final sum is e = lo64[m+1] + hi32[m] (arrays start one limb
// early): value v, generate g, propagate p
__device__ __forceinline__ void carry_limb(const u64 *lo64, const u32 *hi32, long m, u64 *v, bool *g, bool *p)
{
    *g = add_ovf(lo64[m + 1], (u64)hi32[m], v);
    *p = (*v == MPF_MAXL);
}

#define CARRY_V 8  // limbs per thread in the carry kernels (256 threads -> 2048 limbs per block)

// per-thread (generate, propagate) over its CARRY_V contiguous limbs
__device__ __forceinline__ void carry_thread(const u64 *lo64, const u32 *hi32, long m0, long total, bool *G, bool *P)
{
    bool g = false, p = true;
    for (int k = 0; k < CARRY_V; ++k) {
        long m = m0 + k;
        if (m >= total) break;
        u64 v;
        bool gk, pk;
        carry_limb(lo64, hi32, m, &v, &gk, &pk);
        g = gk || (pk && g);
        p = p && pk;
    }
    *G = g;
    *P = p;
}

__global__ __launch_bounds__(256) void k_carry_blocks(const u64 *lo64, const u32 *hi32, long total, u8 *blkG, u8 *blkP)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long m0 = ((long)blockIdx.x * blockDim.x + c.t) * CARRY_V;
    bool G, P;
    carry_thread(lo64, hi32, m0, total, &G, &P);
    u32 co;
    wg_scan<1>(c, G, P, 0, &co, scr);
    // block summary: generate = carry out with cin 0; propagate = every thread propagates
    const u64 allp = __ballot(P);
    __shared__ int pall;
    if (c.t == 0) pall = 1;
    __syncthreads();
    if (c.lane == 0 && allp != ~0ull) pall = 0;
    __syncthreads();
    if (c.t == 0) {
        blkG[blockIdx.x] = (u8)co;
        blkP[blockIdx.x] = (u8)(pall && !co);
    }
}

// single workgroup: carry into every block given the carry `cin` into the first one;
// sum[0] = carry out of the range with cin = 0, sum[1] = every block propagates
__global__ __launch_bounds__(1024) void k_carry_scan(const u8 *blkG, const u8 *blkP, long nblk, u8 *blkC,
                                                     int cin, int *sum)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long per = (nblk + c.nt - 1) / c.nt;
    const long b0 = (long)c.t * per;
    bool g = false, p = true;
    for (long b = b0; b < b0 + per && b < nblk; ++b) {
        g = blkG[b] || (blkP[b] && g);
        p = p && blkP[b];
    }
    u32 co;
    u32 ci = wg_scan<1>(c, g, p, (u32)cin, &co, scr);
    bool run = ci & 1;
    for (long b = b0; b < b0 + per && b < nblk; ++b) {
        blkC[b] = (u8)run;
        run = blkG[b] || (blkP[b] && run);
    }
    if (sum) {
        u32 co0;
        wg_scan<1>(c, g, p, 0, &co0, scr);
        const u64 allp = __ballot(p);
        __shared__ int pall;
        if (c.t == 0) pall = 1;
        __syncthreads();
        if (c.lane == 0 && allp != ~0ull) pall = 0;
        __syncthreads();
        if (c.t == 0) {
            sum[0] = (int)co0;
            sum[1] = pall;
        }
    }
}

__global__ __launch_bounds__(256) void k_carry_apply(const u64 *lo64, const u32 *hi32, long total, const u8 *blkC,
                                                     u64 *r)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long m0 = ((long)blockIdx.x * blockDim.x + c.t) * CARRY_V;
    bool G, P;
    carry_thread(lo64, hi32, m0, total, &G, &P);
    u32 co;
    const u32 ci = wg_scan<1>(c, G, P, blkC[blockIdx.x], &co, scr);
    bool run = ci & 1;
    for (int k = 0; k < CARRY_V; ++k) {
        long m = m0 + k;
        if (m >= total) break;
        u64 v;
        bool gk, pk;
        carry_limb(lo64, hi32, m, &v, &gk, &pk);
        r[m] = v + (run ? 1 : 0);
        run = gk || (pk && run);
        (void)pk;
    }
}

// --------------------------------------------------------------------------
// k_combine1<V>: the whole single-GPU combine in one launch.  Block b owns output limbs
// [256 V b, 256 V (b+1)): it sums the coefficient windows of its limbs (coalesced,
// limb m = base + k 256 + t), resolves its carries locally, and gets its carry-in by a
// decoupled look-back over the blocks before it (flags in `st`, zeroed before the
// launch).  b is a ticket from an atomic counter (st[nblocks]), not blockIdx.x: a block
// only ever waits on blocks that took a smaller ticket, i.e. that are already running,
// whatever order the hardware dispatches workgroups in.
// The flag is the whole message (no data published beside it), so relaxed agent-scope
// atomics suffice: release/acquire would write back / invalidate the XCD's L2 per block.
// Block flag: 0 not ready, 1 aggregate generates, 2 aggregate propagates, 3 aggregate
// kills, 4 / 5 inclusive carry-out 0 / 1.
// --------------------------------------------------------------------------
// limbs per block: 256 V (host: comb_v())

// floor(x / d) for x < 2^52: double quotient, then an exact integer fix-up
__device__ __forceinline__ long udiv_exact(u64 x, u64 d)
{
    long q = (long)((double)x / (double)d);
    while ((u64)q * d > x) --q;
    while ((u64)(q + 1) * d <= x) ++q;
    return q;
}

// coef_ptr for a power-of-two NC (always: NC = 2^floor(depth/2)) and no halo
__device__ __forceinline__ const u64 *coef_ptr2(const CombArgs &a, long k)
{
    const int lg = __builtin_ctz((unsigned)a.NC);
    const long p = (k >> lg) - a.r0;
    const int cc = (int)(k & (a.NC - 1));
    const long slot = (long)(cc >> a.cbb) * a.cbs + p * a.ccb + (cc & (a.ccb - 1));
    return a.dig + (size_t)slot * a.l;
}

__device__ __forceinline__ void comb_limb(const CombArgs &a, long m, u64 *lo, u32 *hi)
{
    const u64 P = (u64)m * 64;
    long klo = (P >= a.N) ? udiv_exact(P - a.N, a.bits1) : 0;
    long khi = udiv_exact(P + 63, a.bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    u64 slo = 0;
    u32 shi = 0;
    for (long k = klo; k <= khi; ++k) {
        const u64 st = (u64)k * a.bits1;
        const u64 *cp = coef_ptr2(a, k);
        u64 v;
        if (st > P) {
            v = cp[0] << (st - P);
        } else {
            const u64 o = P - st;
            const long q = (long)(o >> 6);
            const int s = (int)(o & 63);
            const u64 w0 = (q < a.l) ? cp[q] : 0;
            const u64 w1 = (s && q + 1 < a.l) ? cp[q + 1] : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
        }
        u64 t;
        shi += add_ovf(slo, v, &t);
        slo = t;
    }
    *lo = slo;
    *hi = shi;
}

template <int CB_V>
__global__ __launch_bounds__(256) void k_combine1(CombArgs a, u64 *r, u32 *st)
{
    constexpr int CB_LIMBS = 256 * CB_V;
    __shared__ u64 L[CB_LIMBS];
    __shared__ u32 H[CB_LIMBS + 1];
    __shared__ u64 scr[64];
    __shared__ u32 sh_cin, sh_b;
    const WG c = wg_ctx();
    const long total = a.mcount;
    if (c.t == 0) sh_b = __hip_atomic_fetch_add(&st[gridDim.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const long b = sh_b;   // ticket: every block below b has started
    const long base = b * CB_LIMBS;
    // window sums: lo of limb base + i -> L[i], its carry (hi) -> H[i + 1]
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        const int i = k * 256 + c.t;
        const long m = base + i;
        u64 lo = 0;
        u32 hi = 0;
        if (m < total) comb_limb(a, m, &lo, &hi);
        L[i] = lo;
        H[i + 1] = hi;
    }
    if (c.t == 0) {
        u64 lo = 0;
        u32 hi = 0;
        if (base > 0) comb_limb(a, base - 1, &lo, &hi);
        H[0] = hi;
    }
    __syncthreads();
    // thread t: limbs base + t V .. + V - 1, value v = L + H (H carries the limb below's overflow)
    u64 v[CB_V];
    u32 g = 0, p = 0;
    bool G = false, Pa = true;
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        const int i = c.t * CB_V + k;
        const bool gk = add_ovf(L[i], (u64)H[i], &v[k]);
        const bool pk = v[k] == MPF_MAXL;
        g |= (u32)gk << k;
        p |= (u32)pk << k;
        G = gk || (pk && G);
        Pa = Pa && pk;
    }
    u32 co0;
    wg_scan<1>(c, G, Pa, 0, &co0, scr);
    const bool allp = __syncthreads_and(Pa);
    // look-back (thread 0)
    if (c.t == 0) {
        u32 cin = 0;
        if (b == 0) {
            __hip_atomic_store(&st[0], 4u + co0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const u32 agg = co0 ? 1u : (allp ? 2u : 3u);
            if (agg != 2u) __hip_atomic_store(&st[b], agg == 1u ? 5u : 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(&st[b], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (long j = b - 1;; --j) {
                u32 f;
                while ((f = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
                    __builtin_amdgcn_s_sleep(1);
                if (f >= 4u) { cin = f - 4u; break; }
                if (f == 1u) { cin = 1; break; }
                if (f == 3u) { cin = 0; break; }
            }
            if (agg == 2u) __hip_atomic_store(&st[b], 4u + cin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        sh_cin = cin;
    }
    __syncthreads();
    u32 co;
    const u32 ci = wg_scan<1>(c, G, Pa, sh_cin, &co, scr);
    bool run = ci & 1;
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        L[c.t * CB_V + k] = v[k] + (run ? 1 : 0);
        run = ((g >> k) & 1) || (((p >> k) & 1) && run);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        const long m = base + k * 256 + c.t;
        if (m < total) r[m] = L[k * 256 + c.t];
    }
}
