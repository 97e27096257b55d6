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
// Consecutive limbs per thread (k_combine1<8, KM, true>): thread t sums the windows of limbs
// mA .. mA + 7 (mA = base + 8 t).  The coefficients covering the wave's 512 limbs are found
// once per wave (KM of them at most, host), and every one of them is one word offset and one
// bit shift for all eight limbs: each lane loads the 10 words around its window as five
// aligned 16-B pairs (out-of-range pairs read as zero: before the coefficient, past its l
// words, or a coefficient that does not reach the lane's limbs) and forms each limb with two
// funnel shifts.  Bit b_i = 64 (m0 + mA + i) - k bits1 of c_k is dword 2i + D, shift sh, of the
// loaded pairs (D, sh uniform per coefficient: the lanes' limbs differ by multiples of 8).
// --------------------------------------------------------------------------
typedef u64 cb_v2u __attribute__((ext_vector_type(2)));

template <int D>
__device__ __forceinline__ void comb_acc8(const u32 (&W)[20], int sh, u64 (&lo)[8], u32 (&hi)[8])
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32 x0 = W[2 * i + D], x1 = W[2 * i + D + 1], x2 = W[2 * i + D + 2];
        const u64 v = ((u64)__builtin_amdgcn_alignbit(x2, x1, sh) << 32) | __builtin_amdgcn_alignbit(x1, x0, sh);
        u64 s;
        hi[i] += add_ovf(lo[i], v, &s);
        lo[i] = s;
    }
}

// mW: the wave's first limb (stripe-relative), mA this lane's; total: the stripe's limbs.
// XP: the wave's 257 pairs of a coefficient are loaded coalesced (lane L: pairs L + 64 p) and
// handed to their lanes through the wave's LDS region X (257 x 16 B)
template <int KM, bool XP = false>
__device__ __forceinline__ void comb_thread8(const CombArgs &a, const StripeView &sv, long m0, long mW, long mA,
                                             long total, u64 (&lo)[8], u32 (&hi)[8], cb_v2u *X = nullptr)
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        lo[i] = 0;
        hi[i] = 0;
    }
    if (mW >= total) return;
    const long wl = mW + 512 < total ? mW + 512 : total;
    const u64 P = (u64)(m0 + mW) * 64, Pl = (u64)(m0 + wl - 1) * 64;
    const long klo = (P >= a.N) ? udiv_inv(P - a.N, a.bits1, a.inv_bits1) + 1 : 0;
    long khi = udiv_inv(Pl + 63, a.bits1, a.inv_bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    const long lp = a.l / 2;
    u32 W[KM][20];
    int S2[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {   // every coefficient's pairs requested before any is used
        const long k = klo + j;
        const bool in = k <= khi;
        const i64 o = (i64)(64 * (u64)(m0 + mA) + 64) - (i64)((u64)k * a.bits1);
        const long q = (long)(o >> 6) - 1;   // word of c_k holding limb mA's bit 0 (arithmetic)
        S2[j] = (int)(o & 63) + 64 * (int)(q & 1);
        const long pb = q >> 1;
        const long d = k - sv.kbase;
        const u64 *cp = d < 0 ? sv.chalo + (d + a.H) * (long)a.l : sv.cdig + d * (long)a.l;
        if constexpr (XP) {
            const int L = (int)(mA - mW) >> 3;
            const long pw = pb - 4 * L;   // the wave's first pair
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                const long pp = pw + L + 64 * p;
                cb_v2u x = {0, 0};
                if (in && (p < 4 || L == 0) && pp >= 0 && pp < lp) x = *(const cb_v2u *)(cp + 2 * pp);
                W[j][4 * p] = (u32)x.x;
                W[j][4 * p + 1] = (u32)(x.x >> 32);
                W[j][4 * p + 2] = (u32)x.y;
                W[j][4 * p + 3] = (u32)(x.y >> 32);
            }
        } else {
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                const long pp = pb + p;
                cb_v2u x = {0, 0};
                if (in && pp >= 0 && pp < lp) x = *(const cb_v2u *)(cp + 2 * pp);
                W[j][4 * p] = (u32)x.x;
                W[j][4 * p + 1] = (u32)(x.x >> 32);
                W[j][4 * p + 2] = (u32)x.y;
                W[j][4 * p + 3] = (u32)(x.y >> 32);
            }
        }
    }
    if constexpr (XP) {   // lane L's pairs 4L .. 4L + 4 of the wave's 257
        const int L = (int)(mA - mW) >> 3;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
#pragma unroll
            for (int p = 0; p < 5; ++p)
                if (p < 4 || L == 0) {
                    cb_v2u x;
                    x.x = ((u64)W[j][4 * p + 1] << 32) | W[j][4 * p];
                    x.y = ((u64)W[j][4 * p + 3] << 32) | W[j][4 * p + 2];
                    X[L + 64 * p] = x;
                }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                const cb_v2u x = X[4 * L + p];
                W[j][4 * p] = (u32)x.x;
                W[j][4 * p + 1] = (u32)(x.x >> 32);
                W[j][4 * p + 2] = (u32)x.y;
                W[j][4 * p + 3] = (u32)(x.y >> 32);
            }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (klo + j > khi) break;
        const int s2 = __builtin_amdgcn_readfirstlane(S2[j]);
        const int sh = s2 & 31;
        switch (s2 >> 5) {
        case 0: comb_acc8<0>(W[j], sh, lo, hi); break;
        case 1: comb_acc8<1>(W[j], sh, lo, hi); break;
        case 2: comb_acc8<2>(W[j], sh, lo, hi); break;
        default: comb_acc8<3>(W[j], sh, lo, hi); break;
        }
    }
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
template <int CB_V, int KM, bool CT = false, int NT = 256, bool XP = false>
__global__ __launch_bounds__(NT) void k_combine1(CombArgs a, u64 *r, u32 *st, u32 *allp_out)
{
    constexpr int CB_LIMBS = NT * CB_V;
    static_assert(!CT || (CB_V == 8 && KM > 0), "consecutive limbs per thread: V = 8, a fixed coefficient count");
    static_assert(CT || NT == 256, "the per-limb form runs 256 threads");
    __shared__ u64 L[CB_LIMBS];
    __shared__ u32 H[CT ? NT + 1 : CB_LIMBS + 1];
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
    // thread t: limbs base + t V .. + V - 1, value v = window sum + the limb below's overflow
    u64 v[CB_V];
    u32 g = 0, p = 0;
    bool G = false, Pa = true;
    if constexpr (CT) {
        u64 lo[8];
        u32 hi[8];
        const int t0 = __builtin_amdgcn_readfirstlane(c.t & ~63);
        if constexpr (XP) {
            __shared__ cb_v2u XS[NT / 64][257];
            comb_thread8<KM, true>(a, sv, m0, base + 8L * t0, base + 8L * c.t, total, lo, hi, XS[c.wave]);
        } else {
            comb_thread8<KM>(a, sv, m0, base + 8L * t0, base + 8L * c.t, total, lo, hi);
        }
        H[c.t + 1] = hi[7];
        if (c.t == 0) {
            u64 l0 = 0;
            u32 h0 = 0;
            if (m0 + base > 0 && base < total) comb_limb<KM>(a, sv, m0 + base - 1, &l0, &h0);   // KM >= a limb's count
            H[0] = h0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < CB_V; ++k) {
            const bool real = base + c.t * CB_V + k < total;
            const bool gk = add_ovf(lo[k], (u64)(k ? hi[k - 1] : H[c.t]), &v[k]) && real;
            const bool pk = v[k] == MPF_MAXL || !real;
            g |= (u32)gk << k;
            p |= (u32)pk << k;
            G = gk || (pk && G);
            Pa = Pa && pk;
        }
    } else {
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
        const long m = base + k * NT + c.t;
        if (m < total) rs[m] = L[k * NT + c.t];
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
