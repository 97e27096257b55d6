// combine.hpp -- FFT_combine_bits (mul_fft.c:207-267) on the GPU: limb-parallel
// shifted sums of the canonical coefficients plus a device-wide carry lookahead.
#pragma once
#include "coeff.hpp"

// --------------------------------------------------------------------------
// combine: r = sum_{k < len} c_k 2^(k bits1), c_k < 2^N canonical: per output limb the
// 128-bit sum of the (at most a few) coefficient windows covering it, then the carry chain
// by a decoupled look-back across blocks (k_combine1, one launch).
//
// Stripes.  The product is cut into S stripes of C coefficients: stripe s owns coefficients
// [s C, (s+1) C) and product limbs [ms(s), ms(s+1)), ms(s) = min(total, floor(s C bits1 / 64)),
// ms(S) = total.  A launch combines the stripes s = j G + g for j < nst (one rank's columns
// of the column-sharded multiply: rank g of G holds C consecutive coefficients of every row
// position j, so its stripes are exactly its column-layout rows -- mpfft_shard_combine).
// Each stripe is its own carry chain with carry-in 0; its (generate, propagate) summary lets
// the ranks' stripes be chained afterwards (k_stripe_carry).  The limbs of stripe s only
// read coefficients below (s+1) C (64 ms(s+1) <= (s+1) C bits1), and the H coefficients
// before s C come from `halo`.  The single-GPU combine is one stripe (G = S = 1) over the
// whole coefficient array.
// --------------------------------------------------------------------------
struct CombArgs {
    const u64 *dig;      // canonical coefficients: stripe j's C coefficients at dig + j C l
    int l;
    u64 N, bits1;
    long len;            // number of coefficients j1 + j2 - 1
    long total;          // product limbs
    long C;              // coefficients per stripe
    int G, g;            // stripe j of the launch is stripe j G + g of the product
    long S;              // stripes of the product (the last one ends at limb `total`)
    long bps;            // blocks per stripe
    long SL;             // output stride: stripe j's limbs at r + j SL
    const u64 *halo;     // stripe j's H coefficients before j G + g at halo + j H l (null: none needed)
    int H;
    double inv_bits1;    // 1.0 / bits1 (host), for the window bounds
};

// first product limb of stripe s
__device__ __forceinline__ long stripe_m(const CombArgs &a, long s)
{
    if (s >= a.S) return a.total;
    const long m = (long)(((u64)s * (u64)a.C * a.bits1) >> 6);
    return m < a.total ? m : a.total;
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

// one stripe's view: its coefficients from kbase on at cdig + (k - kbase) l, the H before it
// at chalo + (k - kbase + H) l
struct StripeView {
    const u64 *cdig, *chalo;
    long kbase;
};

// m: global product limb.  KM > 0: at most KM coefficients cover a limb (host:
// ceil((N + 63) / bits1) <= KM), a fixed-trip loop of guarded loads, so a thread's loads for
// all its limbs can be in flight together (the combine is latency-bound otherwise); KM = 0:
// any count.
template <int KM>
__device__ __forceinline__ void comb_limb(const CombArgs &a, const StripeView &sv, long m, u64 *lo, u32 *hi)
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
        const long d = k - sv.kbase;
        const u64 *cp = d < 0 ? sv.chalo + (d + a.H) * (long)a.l : sv.cdig + d * (long)a.l;
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

// --------------------------------------------------------------------------
// k_combine1<V, KM>: nst stripes in one launch, bps blocks of 256 V limbs each.  Block
// (j, b) owns limbs [256 V b, 256 V (b+1)) of stripe j: it sums their coefficient windows
// (coalesced, limb base + k 256 + t), resolves its carries locally, and gets its carry-in by
// a decoupled look-back over the blocks of its stripe before it (flags in `st`, zeroed
// before the launch).  The block index is a ticket from an atomic counter (st[nst bps]), not
// blockIdx.x: a block only ever waits on blocks that took a smaller ticket, i.e. that are
// already running, whatever order the hardware dispatches workgroups in.
// The flag is the whole message (no data published beside it), so relaxed agent-scope
// atomics suffice: release/acquire would write back / invalidate the XCD's L2 per block.
// Block flag: 0 not ready, 1 aggregate generates, 2 aggregate propagates, 3 aggregate
// kills, 4 / 5 inclusive carry-out 0 / 1 (every flag ends at 4 or 5).  Limbs past the
// stripe's end are transparent (propagate), so a stripe's last flag is its carry-out; the
// overflow of its last limb's window sum belongs to the next stripe (its limb ms - 1).
// allp_out (or null): per block, 1 if all its limbs propagate (k_comb_summary).
// --------------------------------------------------------------------------
template <int CB_V, int KM>
__global__ __launch_bounds__(256) void k_combine1(CombArgs a, u64 *r, u32 *st, u32 *allp_out)
{
    constexpr int CB_LIMBS = 256 * CB_V;
    __shared__ u64 L[CB_LIMBS];
    __shared__ u32 H[CB_LIMBS + 1];
    __shared__ u64 scr[64];
    __shared__ u32 sh_cin, sh_b;
    const WG c = wg_ctx();
    if (c.t == 0) sh_b = __hip_atomic_fetch_add(&st[gridDim.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const long tk = sh_b;        // ticket: every block below it has started
    const long j = tk / a.bps, b = tk - j * a.bps;
    const long s = j * a.G + a.g;
    const long m0 = stripe_m(a, s);
    const long total = stripe_m(a, s + 1) - m0;
    StripeView sv;
    sv.kbase = s * a.C;
    sv.cdig = a.dig + j * a.C * (long)a.l;
    sv.chalo = a.halo ? a.halo + j * (long)a.H * a.l : nullptr;
    const long base = b * CB_LIMBS;
    // window sums: lo of limb base + i -> L[i], its carry (hi) -> H[i + 1]
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        const int i = k * 256 + c.t;
        const long m = base + i;
        u64 lo = 0;
        u32 hi = 0;
        if (m < total) comb_limb<KM>(a, sv, m0 + m, &lo, &hi);
        L[i] = lo;
        H[i + 1] = hi;
    }
    if (c.t == 0) {
        u64 lo = 0;
        u32 hi = 0;
        if (m0 + base > 0 && base < total) comb_limb<KM>(a, sv, m0 + base - 1, &lo, &hi);
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
        const bool real = base + i < total;
        const bool gk = add_ovf(L[i], (u64)H[i], &v[k]) && real;
        const bool pk = v[k] == MPF_MAXL || !real;
        g |= (u32)gk << k;
        p |= (u32)pk << k;
        G = gk || (pk && G);
        Pa = Pa && pk;
    }
    u32 co0;
    wg_scan<1>(c, G, Pa, 0, &co0, scr);
    const bool allp = __syncthreads_and(Pa);
    u32 *fl = st + j * a.bps;    // this stripe's flags
    if (allp_out && c.t == 0) allp_out[tk] = allp ? 1u : 0u;
    // look-back (thread 0)
    if (c.t == 0) {
        u32 cin = 0;
        if (b == 0) {
            __hip_atomic_store(&fl[0], 4u + co0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const u32 agg = co0 ? 1u : (allp ? 2u : 3u);
            if (agg != 2u) __hip_atomic_store(&fl[b], agg == 1u ? 5u : 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(&fl[b], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (long q = b - 1;; --q) {
                u32 f;
                while ((f = __hip_atomic_load(&fl[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
                    __builtin_amdgcn_s_sleep(1);
                if (f >= 4u) { cin = f - 4u; break; }
                if (f == 1u) { cin = 1; break; }
                if (f == 3u) { cin = 0; break; }
            }
            if (agg == 2u) __hip_atomic_store(&fl[b], 4u + cin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    u64 *rs = r + j * a.SL;
#pragma unroll
    for (int k = 0; k < CB_V; ++k) {
        const long m = base + k * 256 + c.t;
        if (m < total) rs[m] = L[k * 256 + c.t];
    }
}

// stripe summaries of a k_combine1 launch (one workgroup per stripe j, bps blocks each):
// sum[2 j] = carry out with carry-in 0 (the stripe's last flag), sum[2 j + 1] = every limb
// propagates (all-ones)
__global__ __launch_bounds__(256) void k_comb_summary(const u32 *st, const u32 *allp, long bps, int *sum)
{
    __shared__ int all;
    const long j = blockIdx.x;
    if (threadIdx.x == 0) all = 1;
    __syncthreads();
    int mine = 1;
    for (long b = threadIdx.x; b < bps; b += blockDim.x) mine &= allp[j * bps + b] ? 1 : 0;
    if (!mine) all = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        sum[2 * j] = (int)(st[j * bps + bps - 1] - 4u);
        sum[2 * j + 1] = all;
    }
}

// --------------------------------------------------------------------------
// k_stripe_carry: the carries between stripes.  sums = the G ranks' k_comb_summary outputs
// in rank order ([rank][j][2], nst stripes each): workgroup j finds the carry into stripe
// s = j G + g -- the (generate, propagate) chain of stripes 0 .. s-1 in product order, each
// thread composing a contiguous run of them, thread 0 chaining the runs -- and, when it is
// 1, adds it to the stripe's limbs (r + j SL, `stripe_m` bounds): every all-ones limb wraps to
// zero up to the first one that does not (almost always the first).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stripe_carry(CombArgs a, long nst, const int *sums, u64 *r)
{
    __shared__ u32 gs[256], ps[256];
    __shared__ int cin_sh, stop;
    const long j = blockIdx.x;
    const long s = j * a.G + a.g;
    const int t = threadIdx.x;
    const long per = (s + 255) / 256;
    u32 G = 0, P = 1;
    for (long q = t * per; q < s && q < (t + 1) * per; ++q) {   // stripes q in product order
        const long e = (q % a.G) * nst + q / a.G;
        const u32 gq = (u32)sums[2 * e], pq = (u32)sums[2 * e + 1];
        G = gq | (pq & G);
        P &= pq;
    }
    gs[t] = G;
    ps[t] = P;
    __syncthreads();
    if (t == 0) {
        u32 cin = 0;
        for (int u = 0; u < 256; ++u) cin = gs[u] | (ps[u] & cin);
        cin_sh = (int)cin;
    }
    __syncthreads();
    if (!cin_sh) return;
    const long m0 = stripe_m(a, s), n = stripe_m(a, s + 1) - m0;
    u64 *rs = r + j * a.SL;
    for (long c0 = 0; c0 < n; c0 += 256) {
        const long m = c0 + t;
        const bool ones = m < n && rs[m] == MPF_MAXL;
        const u64 nz = __ballot(!ones && m < n);
        if (t == 0) stop = 1 << 30;
        __syncthreads();
        if ((t & 63) == 0 && nz) atomicMin(&stop, (int)(t + __builtin_ctzll(nz)));
        __syncthreads();
        const int first = stop;   // first non-all-ones limb of this chunk (or none)
        if (m < n && t < first) rs[m] = 0;          // all-ones limbs wrap to zero
        if (m < n && t == first) rs[m] += 1;
        if (first < 256) return;
        __syncthreads();
    }
}
