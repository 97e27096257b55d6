// combine.hpp -- FFT_combine_bits (mul_fft.c:207-267) on the GPU: limb-parallel
// shifted sums of the canonical coefficients plus a device-wide carry lookahead.
#pragma once
#include "coeff.hpp"

// --------------------------------------------------------------------------
// combine: r = sum_{k < len} c_k 2^(k bits1), c_k < 2^N canonical: per output limb the
// 128-bit sum of the (at most a few) coefficient windows covering it, then the carry chain
// by a decoupled look-back across blocks (k_combine1, one launch).
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
    double inv_bits1;    // 1.0 / bits1 (host), for the window bounds
};

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

// floor(x / d) for x < 2^52 from a precomputed inv = fl(1/d): the double product is within
// 1 of x / d, one fix-up each way
__device__ __forceinline__ long udiv_inv(u64 x, u64 d, double inv)
{
    long q = (long)((double)x * inv);
    if ((u64)q * d > x) --q;
    else if ((u64)(q + 1) * d <= x) ++q;
    return q;
}

// m: global product limb (a.m0 + local index); coefficients below kbase come from the halo
// (a rank's combine in the sharded multiply), the rest from the row layout.
// KM > 0: at most KM coefficients cover a limb (host: ceil((N + 63) / bits1) <= KM), a
// fixed-trip loop of guarded loads, so a thread's loads for all its limbs can be in flight
// together (the combine is latency-bound otherwise); KM = 0: any count.
template <int KM>
__device__ __forceinline__ void comb_limb(const CombArgs &a, long m, u64 *lo, u32 *hi)
{
    const u64 P = (u64)m * 64;
    // first coefficient reaching past bit P (k bits1 + N > P) .. last starting below P + 64
    const long klo = (P >= a.N) ? udiv_inv(P - a.N, a.bits1, a.inv_bits1) + 1 : 0;
    long khi = udiv_inv(P + 63, a.bits1, a.inv_bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    u64 slo = 0;
    u32 shi = 0;
    auto window = [&](long k, bool in) {
        // c_k at bit P: o = P - st + 64 in [1, N + 63]; words q = o / 64 - 1 and q + 1 (word -1,
        // before the coefficient, and words >= l read as 0)
        const u64 st = (u64)k * a.bits1;
        const u64 o = P + 64 - st;
        const long q = (long)(o >> 6) - 1;
        const int sb = (int)(o & 63);
        const u64 *cp = k < a.kbase ? a.halo + (size_t)(k - (a.kbase - a.H)) * a.l : coef_ptr2(a, k);
        const u64 w0 = (in && q >= 0 && q < a.l) ? cp[q] : 0;
        const u64 w1 = (in && sb && q + 1 < a.l) ? cp[q + 1] : 0;
        const u64 v = sb ? (w0 >> sb) | (w1 << (64 - sb)) : w0;
        u64 t;
        shi += add_ovf(slo, v, &t);
        slo = t;
    };
    if constexpr (KM > 0) {
#pragma unroll
        for (int j = 0; j < KM; ++j) window(klo + j, klo + j <= khi);
    } else {
        for (long k = klo; k <= khi; ++k) window(k, true);
    }
    *lo = slo;
    *hi = shi;
}

// r[i] = product limb a.m0 + i for i < a.mcount.  A rank of the sharded multiply (m0 > 0)
// starts from carry-in 0 and the overflow of limb m0 - 1; its carry-out with that carry-in
// ends in st[nblocks - 1] (4 + carry) and, when `allp` is given, allp[b] = 1 for every block
// whose limbs all propagate (k_comb_summary turns both into the rank's (generate, propagate)).
template <int CB_V, int KM>
__global__ __launch_bounds__(256) void k_combine1(CombArgs a, u64 *r, u32 *st, u32 *allp_out)
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
        if (m < total) comb_limb<KM>(a, a.m0 + m, &lo, &hi);
        L[i] = lo;
        H[i + 1] = hi;
    }
    if (c.t == 0) {
        u64 lo = 0;
        u32 hi = 0;
        if (a.m0 + base > 0) comb_limb<KM>(a, a.m0 + base - 1, &lo, &hi);
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
    if (allp_out && c.t == 0) allp_out[b] = allp ? 1u : 0u;
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

// rank summary of a k_combine1 launch over nb blocks: sum[0] = carry out with carry-in 0
// (the last block's resolved flag), sum[1] = every limb propagates (all-ones)
__global__ __launch_bounds__(256) void k_comb_summary(const u32 *st, const u32 *allp, long nb, int *sum)
{
    __shared__ int all;
    if (threadIdx.x == 0) all = 1;
    __syncthreads();
    int mine = 1;
    for (long b = threadIdx.x; b < nb; b += blockDim.x) mine &= allp[b] ? 1 : 0;
    if (!mine) all = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        sum[0] = (int)(st[nb - 1] - 4u);
        sum[1] = all;
    }
}

// r[0 .. n) += 1 (the carry into a rank's limb range from the ranks below): one workgroup
// walks 256-limb chunks until the first limb that is not all-ones (the first, almost always)
__global__ __launch_bounds__(256) void k_carry_in(u64 *r, long n)
{
    __shared__ int stop;
    for (long c0 = 0; c0 < n; c0 += 256) {
        const long m = c0 + threadIdx.x;
        const bool ones = m < n && r[m] == MPF_MAXL;
        const u64 nz = __ballot(!ones && m < n);
        if (threadIdx.x == 0) stop = 1 << 30;
        __syncthreads();
        if ((threadIdx.x & 63) == 0 && nz) atomicMin(&stop, (int)(threadIdx.x + __builtin_ctzll(nz)));
        __syncthreads();
        const int first = stop;   // first non-all-ones limb of this chunk (or none)
        if (m < n && (int)threadIdx.x < first) r[m] = 0;          // all-ones limbs wrap to zero
        if (m < n && (int)threadIdx.x == first) r[m] += 1;
        if (first < 256) return;
        __syncthreads();
    }
}
