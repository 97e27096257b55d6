// fold.hpp -- the final scaling and canonicalisation folded away.
//
// The reference scales every coefficient by 2^-(depth+1) and normalises it
// (mpn_div_2expmod_2expp1 + mpn_normmod_2expp1 in the loop at mul_fft.c:3256-3260) before
// FFT_combine_bits (:3261-3262, :207-267) adds the coefficients at offsets k bits1.  Here,
// on the single-GPU truncated plans, that loop is not a pass of its own:
//   - the 2^-(depth+1) rides in the last inverse row pass's MFA un-twiddle (one more exponent in
//     the rotation that pass applies anyway; the inverse column transform is linear);
//   - the truncated inverse's deferred top-level doubling (rows [dbl_lo, dbl_hi)) is a one-bit
//     shift of those coefficients' windows in the combine (s_k = 1);
//   - the coefficients stay in the passes' reduced form (limbs, {-1,0,+1} carry masks, carry
//     limb), which the combine reads directly: carries are +-2^(64 i) terms at their limbs, and
//     the wrap to the canonical residue is one small integer per coefficient, m_k = floor(X_k / p)
//     for X_k = 2^s_k V_k, p = 2^N + 1, so that c_k = X_k - m_k p = 2^s_k L_k + A_k 2^N + B_k
//     with A_k = 2^s_k (top_k + carry out of the last limb) - m_k and B_k = -m_k (k_cmeta);
//   - the combine's carries become signed ({-1, 0, +1}), chained as transfer functions
//     (k_combine_red): per limb c -> floor((u + c) / 2^64) + g, composed by a wave scan, a
//     workgroup scan and the decoupled look-back of k_combine1.
// This is what the reference's TODO asks for (TODO:53-59: "combine just a single coefficient at
// a time so that cache locality can be maintained for the MFA IFFT's") -- no pass over the
// coefficients between the inverse transform and the combine.
#pragma once
#include "combine.hpp"

// ---- carry transfer functions ------------------------------------------------------------
// A function of the incoming carry c in {-1, 0, 1} to the outgoing one, as three 2-bit fields
// (value + 1 at bits 2 (c + 1)).  Limb with local carry g and value u (mod 2^64) before the
// carry-in: f(c) = g + [c == 1 and u == 2^64 - 1] - [c == -1 and u == 0] (|g + ...| <= 1 as long
// as the limb's signed overflow is small: g = 1 leaves u small, g = -1 leaves u large).
#define CF_ID 0x24u
__host__ __device__ __forceinline__ u32 cf_make(int g, u64 u)
{
    const int fm = g - (u == 0 ? 1 : 0), fp = g + (u == MPF_MAXL ? 1 : 0);
    return (u32)(fm + 1) | ((u32)(g + 1) << 2) | ((u32)(fp + 1) << 4);
}
__host__ __device__ __forceinline__ int cf_apply(u32 f, int c) { return (int)((f >> (2 * (c + 1))) & 3u) - 1; }
// f first, then g
__host__ __device__ __forceinline__ u32 cf_then(u32 f, u32 g)
{
    u32 h = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) h |= ((g >> (2 * ((f >> (2 * c)) & 3u))) & 3u) << (2 * c);
    return h;
}
__host__ __device__ __forceinline__ bool cf_const(u32 f) { return (f & 3u) == ((f >> 2) & 3u) && (f & 3u) == ((f >> 4) & 3u); }

// inclusive scan over the 64 lanes of a wave in lane order (lane 0's function applied first)
__device__ __forceinline__ u32 cf_wave_scan(u32 f, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 o = (u32)__shfl_up((int)f, d);
        if (lane >= d) f = cf_then(o, f);
    }
    return f;
}

// x 2^b (b < 64, x a small signed integer) added to the 128-bit signed accumulator (lo, hi)
template <typename HI>
__device__ __forceinline__ void acc_signed(u64 &lo, HI &hi, i64 x, int b)
{
    const u64 v = (u64)x << b;
    const i64 h = b ? (x >> (64 - b)) : (x < 0 ? -1 : 0);
    u64 t;
    const bool c = add_ovf(lo, v, &t);
    lo = t;
    hi += (HI)((int)h + (c ? 1 : 0));   // u32 hi: two's complement
}

struct FoldArgs {
    const u64 *dig;      // coefficient k at dig + k l (reduced form, single-GPU natural slot order)
    const u64 *cb;       // its carry masks at cb + k cbw
    const int *top;      // its carry limb
    int *meta;           // k_cmeta's output: A_k (low 16 bits) and B_k (high 16 bits), signed
    int l, cbw;
    u64 N, bits1;
    long len, total;     // coefficients, product limbs
    int lbC;             // coefficient k is in row k >> lbC
    int dbl_lo, dbl_hi;  // rows whose coefficients are doubled (s_k = 1)
    long bps;            // combine blocks
    double inv_bits1;
};

__device__ __forceinline__ int fold_s(const FoldArgs &a, long k)
{
    const long row = k >> a.lbC;
    return row >= a.dbl_lo && row < a.dbl_hi ? 1 : 0;
}
__device__ __forceinline__ int meta_A(int m) { return (int)(short)(m & 0xffff); }
__device__ __forceinline__ int meta_B(int m) { return m >> 16; }

// ---- k_cmeta: A_k, B_k per coefficient ------------------------------------------------------
// Resolving the carries of L_k (its limbs plus carries) gives resolved limbs R_i and the carry
// out Lhi; X = 2^s V = Xlo + Xhi 2^N with Xlo = (2^s sum R_i 2^(64 i)) mod 2^N and
// Xhi = 2^s (top + cl + Lhi) + s bit (N - 1) of R.  m = Xhi, minus 1 if Xlo < Xhi, plus 1 if
// Xlo - Xhi >= p.  Fast path, one lane per coefficient (64 per wave): when limb l - 2 (with its
// carry-in) is neither 0 nor all ones it absorbs any carry from below, which fixes R_(l-1), Lhi and
// (for s = 1) the top bit of R_(l-2); if Xlo's top limb is then neither 0 nor all ones, Xlo - Xhi
// lies in [0, p) for any small Xhi and m = Xhi (and with a zero top limb too when Xhi <= 0, with
// an all-ones one when Xhi >= -1).  Otherwise (adversarial inputs: runs of 0 or all-ones limbs)
// the whole wave resolves that coefficient (cmeta_full).
template <int NL>   // NL = l / 64 limbs per lane held in registers (one round trip); 0: runtime l, batches of 8
__device__ int cmeta_full(const FoldArgs &a, long k, int lane)
{
    // lane L resolves limbs [L nl, (L + 1) nl): its limbs' composite transfer function (one
    // sequential sweep), a wave scan for the carries into the lanes, a second sweep for the
    // resolved limbs
    const int l = a.l, nl = NL ? NL : l >> 6;
    const u64 *d = a.dig + k * (long)l;
    const u64 *cb = a.cb + k * (long)a.cbw;
    const int s = fold_s(a, k);
    const int bl = l - 1;
    const int cl = (int)((cb[2 * (bl >> 6)] >> (bl & 63)) & 1) - (int)((cb[2 * (bl >> 6) + 1] >> (bl & 63)) & 1);
    const int T0 = a.top[k] + cl;
    const int i0 = lane * nl;
    // the lane's limbs 8 at a time (16-B loads, all in flight), with their carry-ins: mask bits
    // i - 1 (the lane's limbs lie in one 64-limb mask row; limb i0's carry-in is bit 63 of the
    // row below)
    const int W = i0 >> 6;
    const cb_v2u mrow = *(const cb_v2u *)(cb + 2 * W);
    const cb_v2u mprev = W ? *(const cb_v2u *)(cb + 2 * W - 2) : cb_v2u{0, 0};
    auto cin_of = [&](int i) -> int {
        if (i == 0) return 0;
        const int b = i - 1;
        const cb_v2u m = (b >> 6) == W ? mrow : mprev;
        return (int)((m.x >> (b & 63)) & 1) - (int)((m.y >> (b & 63)) & 1);
    };
    auto batch = [&](int i, u64 (&x)[8]) {
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
            const cb_v2u v = *(const cb_v2u *)(d + i + q);
            x[q] = v.x;
            x[q + 1] = v.y;
        }
    };
    auto limb = [&](int i, u64 x, u64 &u) -> int {   // limb i with its carry-in; returns its local carry
        const int c = cin_of(i);
        u = x + (u64)(i64)c;
        return (c == 1 && x == MPF_MAXL) ? 1 : (c == -1 && x == 0) ? -1 : 0;
    };
    u32 F = CF_ID;
    u64 xa[NL ? NL : 1];
    if constexpr (NL > 0) {   // every limb of the lane requested at once, kept for the second sweep
#pragma unroll
        for (int q = 0; q < NL; q += 2) {
            const cb_v2u v = *(const cb_v2u *)(d + i0 + q);
            xa[q] = v.x;
            xa[q + 1] = v.y;
        }
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            u64 u;
            const int g = limb(i0 + q, xa[q], u);
            F = cf_then(F, cf_make(g, u));
        }
    } else {
        for (int i = i0; i < i0 + nl; i += 8) {
            u64 x[8];
            batch(i, x);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                u64 u;
                const int g = limb(i + q, x[q], u);
                F = cf_then(F, cf_make(g, u));
            }
        }
    }
    const u32 I = cf_wave_scan(F, lane);
    u32 E = (u32)__shfl_up((int)I, 1);
    if (lane == 0) E = CF_ID;
    int c = cf_apply(E, 0);   // carry into limb i0 (none into limb 0)
    bool allz = true, allo = true;
    u64 Rfirst = 0, R = 0, prev = 0;
    auto resolve = [&](int i, u64 xv) {   // limb i (>= i0) with the carry c from below
        u64 u;
        const int g = limb(i, xv, u);
        R = u + (u64)(i64)c;
        c = cf_apply(cf_make(g, u), c);
        if (i == i0) {
            Rfirst = R;
        } else {
            const u64 X = s ? (R << 1) | (prev >> 63) : R;   // Xlo's limb i (>= 1)
            allz = allz && X == 0;
            allo = allo && X == MPF_MAXL;
        }
        prev = R;
    };
    if constexpr (NL > 0) {
#pragma unroll
        for (int q = 0; q < NL; ++q) resolve(i0 + q, xa[q]);
    } else {
        for (int i = i0; i < i0 + nl; i += 8) {
            u64 x[8];
            batch(i, x);
#pragma unroll
            for (int q = 0; q < 8; ++q) resolve(i + q, x[q]);
        }
    }
    u64 pl = __shfl_up(R, 1);   // the limb below i0
    if (lane == 0) pl = 0;
    const u64 Xf = s ? (Rfirst << 1) | (pl >> 63) : Rfirst;
    if (lane) {
        allz = allz && Xf == 0;
        allo = allo && Xf == MPF_MAXL;
    }
    allz = __ballot(!allz) == 0;
    allo = __ballot(!allo) == 0;
    const u64 x0 = __shfl(Xf, 0);
    const u64 Rtop = __shfl(R, 63);
    const int Lhi = __shfl(c, 63);
    const int Xhi = (T0 + Lhi) * (1 << s) + (s ? (int)(Rtop >> 63) : 0);
    int m = Xhi;
    if (allz && Xhi > 0 && x0 < (u64)Xhi) m -= 1;                        // Xlo < Xhi
    if (allo && Xhi <= -2 && ~x0 <= (u64)(-(i64)Xhi - 2)) m += 1;        // Xlo - Xhi >= p
    return T0 * (1 << s) - m;   // A; B = -m
}

__device__ __forceinline__ void cmeta_store(const FoldArgs &a, long k, int A, int B)
{
    a.meta[k] = (A & 0xffff) | (int)((unsigned)B << 16);
}

template <int NL>   // l / 64 for l = 1024 / 2048 / 4096 (the slow path's limbs per lane in registers), 0 any l
__global__ __launch_bounds__(256) void k_cmeta(FoldArgs a)
{
    const int lane = threadIdx.x & 63;
    const long kw = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;   // the wave's first coefficient
    const long k = kw + lane;
    const int l = a.l;
    bool done = true;
    if (k < a.len) {
        const u64 *d = a.dig + k * (long)l;
        const cb_v2u x = *(const cb_v2u *)(d + l - 2);                          // limbs l - 2, l - 1
        const cb_v2u mw = *(const cb_v2u *)(a.cb + k * (long)a.cbw + a.cbw - 2);   // mask bits l - 64 .. l - 1
        const int top = a.top[k];
        const int s = fold_s(a, k);
        auto bit = [&](int b) -> int { return (int)((mw.x >> (b & 63)) & 1) - (int)((mw.y >> (b & 63)) & 1); };
        const int c1 = bit(l - 3), c2 = bit(l - 2), cl = bit(l - 1);   // carries into l - 2, l - 1, out of l - 1
        const u64 u1 = x.x + (u64)(i64)c1, u2 = x.y + (u64)(i64)c2;
        const int g1 = (c1 == 1 && x.x == MPF_MAXL) ? 1 : (c1 == -1 && x.x == 0) ? -1 : 0;
        const int g2 = (c2 == 1 && x.y == MPF_MAXL) ? 1 : (c2 == -1 && x.y == 0) ? -1 : 0;
        // limb l - 2 absorbs any carry-in (u1 not 0 / all ones): its carry-out is g1, and its top bit
        // is that of u1 + any of -1, 0, 1 unless u1 sits at 2^63 -+ 1
        done = u1 != 0 && u1 != MPF_MAXL && (!s || ((u1 - 1) >> 63) == ((u1 + 1) >> 63));
        if (done) {
            const u64 R2 = u2 + (u64)(i64)g1;
            const int Lhi = cf_apply(cf_make(g2, u2), g1);
            const u64 xt = s ? (R2 << 1) | (u1 >> 63) : R2;
            const int T0 = top + cl;
            const int m = (T0 + Lhi) * (1 << s) + (s ? (int)(R2 >> 63) : 0);   // Xhi
            // Xlo < Xhi needs Xhi > 0 and Xlo's top limb 0; Xlo - Xhi >= p needs Xhi <= -2 and
            // that limb all ones: otherwise m = Xhi exactly (small coefficients -- the product's
            // ends -- have a zero top limb, but Xhi <= 0 unless their carry limb is positive)
            done = (xt != 0 || m <= 0) && (xt != MPF_MAXL || m >= -1);
            if (done) cmeta_store(a, k, T0 * (1 << s) - m, -m);
        }
    }
    u64 rest = __ballot(!done);
    while (rest) {   // wave-uniform
        const int ln = __builtin_ctzll(rest);
        rest &= rest - 1;
        const long kk = kw + ln;
        const int A = cmeta_full<NL>(a, kk, lane);
        if (lane == 0) {
            const int s = fold_s(a, kk);
            const u64 *cb = a.cb + kk * (long)a.cbw;
            const int bl = l - 1;
            const int cl = (int)((cb[2 * (bl >> 6)] >> (bl & 63)) & 1) - (int)((cb[2 * (bl >> 6) + 1] >> (bl & 63)) & 1);
            const int T0 = a.top[kk] + cl;
            cmeta_store(a, kk, A, A - T0 * (1 << s));
        }
    }
}

// ---- the reduced-form combine --------------------------------------------------------------
// per output limb: the windows of the coefficients covering it (shifted by s_k), their carries,
// and the A_k 2^N, B_k terms landing in it, as a 128-bit signed sum (lo, hi)

// one limb (the limb below a block, for its overflow): every load of it -- KM coefficients'
// window words and mask words, the A / B terms' meta words -- issued before any is used (a
// fixed-trip loop of guarded loads, as comb_limb: thread 0 runs this while the block waits)
// timing probes (A/B builds only, wrong products): bit 0 no limb below the block (fold_limb), bit 1 no
// carries from the masks, bit 2 no A / B terms
#ifndef FOLD_PERSIST
#define FOLD_PERSIST 1   // 0 (A/B builds): one workgroup per ticket, a grid of bps blocks
#endif
#ifndef FOLD_PROBE
#define FOLD_PROBE 0
#endif
template <int KM>
__device__ void fold_limb(const FoldArgs &a, long m, u64 *plo, int *phi)
{
    const u64 P = (u64)m * 64;
    const long klo = (P >= a.N + 1) ? udiv_inv(P - a.N - 1, a.bits1, a.inv_bits1) + 1 : 0;
    long khi = udiv_inv(P + 63, a.bits1, a.inv_bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    const long kB = P ? udiv_inv(P - 1, a.bits1, a.inv_bits1) + 1 : 0;
    const bool hasB = kB < a.len && (u64)kB * a.bits1 < P + 64;
    const long kA = P <= a.N ? 0 : udiv_inv(P - a.N - 1, a.bits1, a.inv_bits1) + 1;
    const u64 pa = (u64)kA * a.bits1 + a.N;
    const bool hasA = P + 63 >= a.N && kA < a.len && pa >= P && pa < P + 64;
    const int mB = hasB ? a.meta[kB] : 0, mA = hasA ? a.meta[kA] : 0;
    u64 w0[KM], w1[KM], cp0[KM], cn0[KM];
    int sbv[KM], qqv[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const long k = klo + j;
        const bool in = k <= khi;
        const int s = in ? fold_s(a, k) : 0;
        const i64 o = (i64)(P + 64) - (i64)((u64)k * a.bits1) - s;
        const long q = (long)(o >> 6) - 1;
        const int sb = (int)(o & 63);
        const u64 *cp = a.dig + k * (long)a.l;
        w0[j] = (in && q >= 0 && q < a.l) ? cp[q] : 0;
        w1[j] = (in && sb && q + 1 >= 0 && q + 1 < a.l) ? cp[q + 1] : 0;
        const long qq = q + (sb ? 1 : 0);   // the limb whose bit 0 lands in this window
        const bool hc = in && qq >= 1 && qq <= a.l - 1;
        const long bb = hc ? qq - 1 : 0;
        const u64 *cc = a.cb + k * (long)a.cbw + 2 * (bb >> 6);
        cp0[j] = hc ? cc[0] >> (bb & 63) : 0;
        cn0[j] = hc ? cc[1] >> (bb & 63) : 0;
        sbv[j] = sb;
        qqv[j] = (int)(bb & 63);
    }
    u64 lo = 0;
    int hi = 0;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int sb = sbv[j];
        const u64 v = sb ? (w0[j] >> sb) | (w1[j] << (64 - sb)) : w0[j];
        u64 t;
        hi += add_ovf(lo, v, &t) ? 1 : 0;
        lo = t;
        const int dd = (int)(cp0[j] & 1) - (int)(cn0[j] & 1);
        if (dd) acc_signed(lo, hi, dd, (64 - sb) & 63);
    }
    if (hasB) acc_signed(lo, hi, meta_B(mB), (int)((u64)kB * a.bits1 - P));
    if (hasA) acc_signed(lo, hi, meta_A(mA), (int)(pa - P));
    *plo = lo;
    *phi = hi;
}

// limbs mA .. mA + 7 of this lane (mW: the wave's first limb): comb_thread8's coalesced window
// loads (the wave's 257 pairs of a coefficient through its LDS region X); the carry-mask words the
// wave's limbs need (nine 16-B pairs per coefficient, lanes 0-8) the same way through MS, in flight
// with the window words; then the A / B terms of the (at most KM) coefficients landing here.
// (lo, hi) per limb: the 128-bit signed sum, hi in two's complement
template <int KM>
__device__ __forceinline__ void fold_thread8(const FoldArgs &a, long mW, long mA, long total, u64 (&lo)[8], u32 (&hi)[8],
                                             cb_v2u *X, cb_v2u (*MS)[9])
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        lo[i] = 0;
        hi[i] = 0;
    }
    if (mW >= total) return;
    const long wl = mW + 512 < total ? mW + 512 : total;
    const u64 P = (u64)mW * 64, Pl = (u64)(wl - 1) * 64;
    const long klo = (P >= a.N + 1) ? udiv_inv(P - a.N - 1, a.bits1, a.inv_bits1) + 1 : 0;
    long khi = udiv_inv(Pl + 63, a.bits1, a.inv_bits1);
    if (khi > a.len - 1) khi = a.len - 1;
    const long lp = a.l / 2, nmw = a.l / 64;
    const int L = (int)(mA - mW) >> 3;
    u32 W[KM][20];
    int S2[KM], mt[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {   // every coefficient's pairs and mask words requested before any is used
        const long k = klo + j;
        const bool in = k <= khi;
        mt[j] = in ? a.meta[k] : 0;   // k wave-uniform
        const int s = in ? fold_s(a, k) : 0;
        const i64 o = (i64)(64 * (u64)mA + 64) - (i64)((u64)k * a.bits1) - s;
        const long q = (long)(o >> 6) - 1;   // word of c_k holding limb mA's bit 0 (arithmetic)
        const int r = (int)(o & 63);
        S2[j] = r + 64 * (int)(q & 1);
        const long pb = q >> 1;
        const u64 *cp = a.dig + k * (long)a.l;
        const long pw = pb - 4 * L;   // the wave's first pair
        // the carries into limbs q + i + [r > 0] of c_k are mask bits e0 + i: the wave's lanes span
        // e0 .. e0 + 511 + 8 from lane 0's, mask words W0 .. W0 + 8 -- loaded by lanes 1-9 into
        // the registers of the wave's 257th pair, which only lane 0 holds
        const long e0w = q - 8 * L + (r ? 1 : 0) - 1;
        const long mwi = (e0w >> 6) + L - 1;
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            const long pp = pw + L + 64 * p;
            cb_v2u x = {0, 0};
            if (p < 4 || L == 0) {
                if (in && pp >= 0 && pp < lp) x = *(const cb_v2u *)(cp + 2 * pp);
            } else if (L <= 9) {
                if (in && mwi >= 0 && mwi < nmw) x = *(const cb_v2u *)(a.cb + k * (long)a.cbw + 2 * mwi);
            }
            W[j][4 * p] = (u32)x.x;
            W[j][4 * p + 1] = (u32)(x.x >> 32);
            W[j][4 * p + 2] = (u32)x.y;
            W[j][4 * p + 3] = (u32)(x.y >> 32);
        }
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) {   // lane L's pairs 4L .. 4L + 4 of the wave's 257
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            cb_v2u x;
            x.x = ((u64)W[j][4 * p + 1] << 32) | W[j][4 * p];
            x.y = ((u64)W[j][4 * p + 3] << 32) | W[j][4 * p + 2];
            if (p < 4 || L == 0) X[L + 64 * p] = x;
            else if (L <= 9) MS[j][L - 1] = x;
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
    // the carries (at bit (64 - r) mod 64 of limb i) and the A_k 2^N, B_k terms: coefficient k's
    // B at bit k bits1 and A at k bits1 + N lie in this wave's bits only for k in [klo, khi]
    const u64 PL = (u64)mA * 64, PW = (u64)mW * 64;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const long k = klo + j;
        if (k > khi) break;
        const int s = fold_s(a, k);
        const u64 kb = (u64)k * a.bits1;
        const int r = (int)((PL + 64 - kb - s) & 63);
        u32 cb;   // 8 + 8 bits of + / - carries into the lane's limbs (their mask words in MS since the handoff)
        {
            const i64 o = (i64)(64 * (u64)mA + 64) - (i64)kb - s;
            const long q = (long)(o >> 6) - 1;
            const long e0 = q + ((o & 63) ? 1 : 0) - 1;
            const long e0w = e0 - 8 * L;
            const int i0 = (int)((e0 >> 6) - (e0w >> 6));
            const cb_v2u m0 = MS[j][i0], m1 = MS[j][i0 < 8 ? i0 + 1 : 8];
            const int sh = (int)(e0 & 63);
            const u64 pbits = sh ? (m0.x >> sh) | (m1.x << (64 - sh)) : m0.x;
            const u64 nbits = sh ? (m0.y >> sh) | (m1.y << (64 - sh)) : m0.y;
            // bits e0 + i valid for 0 <= e0 + i <= l - 2
            const long lb = e0 < 0 ? -e0 : 0, ub = (long)a.l - 1 - e0;
            const u32 vm = (lb >= 8 || ub <= 0) ? 0u : ((ub >= 8 ? 0xffu : (1u << ub) - 1u) & ~((1u << lb) - 1u));
            cb = ((u32)pbits & vm) | (((u32)nbits & vm) << 8);
        }
        if ((FOLD_PROBE & 2) == 0 && __ballot(cb != 0)) {   // branch-free per limb: d 2^shc with d in {-1, 0, 1} (shc wave-uniform)
            const int shc = (64 - r) & 63;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int dd = (int)((cb >> i) & 1) - (int)((cb >> (8 + i)) & 1);
                u64 t;
                const bool c = add_ovf(lo[i], (u64)(i64)dd << shc, &t);
                lo[i] = t;
                hi[i] += (u32)((c ? 1 : 0) - (dd < 0 ? 1 : 0));
            }
        }
        // A_k 2^N and B_k: bits k bits1 + N and k bits1, N (> a wave's 512 limbs) apart, so a wave
        // holds at most one of the two, in one lane, at a wave-uniform position: the term is formed
        // on the scalar side and added to the limb it names by a uniform switch (the per-lane select
        // over all 8 limbs cost 24 us of C3's combine, profiles/r06/probes.txt)
        const int mu = __builtin_amdgcn_readfirstlane(mt[j]);
        const int vB = meta_B(mu), vA = meta_A(mu);
        const u64 ka = kb + a.N;
        const bool inB = vB && kb >= PW && kb < PW + 32768, inA = vA && ka >= PW && ka < PW + 32768;
        if (inB || inA) {
            const i64 x = inB ? vB : vA;
            const u64 bp = (inB ? kb : ka) - PW;   // bit within the wave's 512 limbs
            const int Ls = (int)(bp >> 9), li = __builtin_amdgcn_readfirstlane((int)((bp >> 6) & 7)), b = (int)(bp & 63);
            const u64 xl = L == Ls ? (u64)x << b : 0;
            const u32 xh = L == Ls ? (u32)(b ? (x >> (64 - b)) : (x < 0 ? -1 : 0)) : 0u;
            auto add_at = [&](int i) {
                u64 t;
                const bool c = add_ovf(lo[i], xl, &t);
                lo[i] = t;
                hi[i] += xh + (c ? 1u : 0u);
            };
            switch (li) {
            case 0: add_at(0); break;
            case 1: add_at(1); break;
            case 2: add_at(2); break;
            case 3: add_at(3); break;
            case 4: add_at(4); break;
            case 5: add_at(5); break;
            case 6: add_at(6); break;
            default: add_at(7); break;
            }
        }
    }
}

// k_combine_red<KM, NT>: the product from the reduced-form coefficients, blocks of 8 NT limbs
// (8 consecutive limbs per thread), one launch: window sums, a signed carry chain per block as
// transfer functions (wave scan + workgroup scan), and the decoupled look-back of k_combine1 over
// ticket-ordered blocks.  Flags: 0 not ready, 8 + (carry out + 1) inclusive, 16 + f the block's
// transfer function f (not yet inclusive); st zeroed before the launch, st[bps] the ticket counter.
template <int KM, int NT>
__global__ __launch_bounds__(NT, KM <= 3 ? 2048 / NT : 1) void k_combine_red(FoldArgs a, u64 *r, u32 *st)
{
    constexpr int V = 8, CB = NT * V, NW = NT / 64;
    __shared__ u64 Lx[CB];
    __shared__ int H[NT + 1];
    __shared__ u32 WF[NW];
    __shared__ cb_v2u XS[NW][257];
    __shared__ cb_v2u MS[NW][KM][9];
    __shared__ u32 sh_b;
    __shared__ int sh_cin;
    const long nb = a.bps;   // st[nb]: the ticket counter
    if (threadIdx.x == 0) sh_b = __hip_atomic_fetch_add(&st[nb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    // persistent (FOLD_PERSIST: a grid of about the resident block count): a workgroup takes tickets
    // until they run out, the next one requested at the start of this one's work so its round trip
    // hides under the loads; each ticket's work is the one-block body below
    for (;;) {
        // the thread index as an opaque value per ticket: what derives from it is recomputed, not
        // kept live across the loop (hoisted, it spilled 44 B per lane)
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        const int lane = t & 63, wave = t >> 6;
        const long b = sh_b;   // ticket: every block below it has started
        if (b >= nb) break;   // workgroup-uniform
        u32 nxt = 0;
        if (t == 0) nxt = __hip_atomic_fetch_add(&st[nb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const long total = a.total;
        const long base = b * CB;
        u64 lo[8];
        u32 hu[8];
        const int t0 = __builtin_amdgcn_readfirstlane(t & ~63);
        fold_thread8<KM>(a, base + 8L * t0, base + 8L * t, total, lo, hu, XS[wave], MS[wave]);
        int hi[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) hi[k] = (int)hu[k];
        H[t + 1] = hi[7];
        if (t == 0) {
            u64 l0 = 0;
            int h0 = 0;
            if ((FOLD_PROBE & 1) == 0 && base > 0 && base < total) fold_limb<KM>(a, base - 1, &l0, &h0);
            H[0] = h0;
        }
        __syncthreads();
        u64 u[8];
        u32 gk = 0;   // limb k's local carry + 1 at bits 2k (3: past the end, transparent)
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const bool real = base + 8L * t + k < total;
            const int hin = k ? hi[k - 1] : H[t];
            const u64 v = lo[k] + (u64)(i64)hin;
            const int g = hin >= 0 ? (v < lo[k] ? 1 : 0) : (v > lo[k] ? -1 : 0);
            u[k] = v;
            gk |= (real ? (u32)(g + 1) : 3u) << (2 * k);
        }
        auto fk = [&](int k) -> u32 {
            const u32 gq = (gk >> (2 * k)) & 3u;
            return gq == 3u ? CF_ID : cf_make((int)gq - 1, u[k]);
        };
        // the thread's composite, last limb first: a limb that neither is 0 nor all ones maps every
        // carry-in to its own carry, so the composite almost always stops at limb 7
        u32 F = fk(7);
#pragma unroll
        for (int k = 6; k >= 0; --k)
            if (!cf_const(F)) F = cf_then(fk(k), F);
        u32 I, Ex;
        if (__ballot(!cf_const(F)) == 0) {   // every lane constant: lane L's carry-in is lane L - 1's carry-out
            I = F;
            Ex = (u32)__shfl_up((int)F, 1);
        } else {
            I = cf_wave_scan(F, lane);
            Ex = (u32)__shfl_up((int)I, 1);
        }
        if (lane == 0) Ex = CF_ID;
        if (lane == 63) WF[wave] = I;
        __syncthreads();
        // the composites of the waves below (Wp) and of the block (Fb); a constant wave function
        // overrides everything before it, the common case
        u32 Wp = CF_ID, Fb = CF_ID;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const u32 f = WF[w];
            const u32 nb = cf_const(f) ? f : cf_then(Fb, f);
            if (w < wave) Wp = nb;
            Fb = nb;
        }
        if (t == 0) {
            int cin = 0;
            if (b == 0) {
                __hip_atomic_store(&st[0], 9u + (u32)cf_apply(Fb, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const bool cst = cf_const(Fb);
                __hip_atomic_store(&st[b], cst ? 9u + (u32)cf_apply(Fb, 0) : 16u + Fb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                u32 acc = CF_ID;
                for (long q = b - 1;; --q) {
                    u32 f;
                    while ((f = __hip_atomic_load(&st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
                        __builtin_amdgcn_s_sleep(1);
                    if (f < 16u) {
                        cin = cf_apply(acc, (int)f - 9);
                        break;
                    }
                    acc = cf_then(f - 16u, acc);
                }
                if (!cst) __hip_atomic_store(&st[b], 9u + (u32)cf_apply(Fb, cin), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            sh_cin = cin;
        }
        __syncthreads();
        int c = cf_apply(cf_then(Wp, Ex), sh_cin);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            Lx[t * V + k] = u[k] + (u64)(i64)c;
            const int gq = (int)((gk >> (2 * k)) & 3u) - 1;   // 2: past the end (transparent)
            c = gq == 2 ? c : gq + (c == 1 && u[k] == MPF_MAXL) - (c == -1 && u[k] == 0);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const long m = base + k * NT + t;
            if (m < total) r[m] = Lx[k * NT + t];
        }
        __syncthreads();   // every read of this ticket's LDS done
        if (t == 0) sh_b = nxt;
        __syncthreads();
    }
}
