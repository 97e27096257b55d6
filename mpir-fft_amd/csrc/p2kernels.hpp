// p2kernels.hpp -- k_pw2: the nested negacyclic pointwise of pkernels.hpp (SURVEY 8f rank 1:
// FFT_mulmod_2expp1 / fft_mulmod_2expp1, mul_fft.c:2998-3167) with TWO threads per piece.
//
// Why: k_pwss keeps a whole inner-ring value (M limbs) per thread, so a workgroup of K threads
// needs ~160 VGPRs (C3) to ~210 (C4) and the kernel runs 2-3 waves per SIMD, latency-bound
// (profiles/pmc_C3.json: VALU 0.47 issue / LDS 0.33, the rest waiting).  Here lanes 2i and
// 2i+1 hold the low and high half of piece i (HL = M/2 limbs each):
//   * the value of a piece is  (-1)^S (L_lo + (L_hi + C) X + T 2^N'),  X = 2^(64 HL); T (the
//     top) and C (a carry of the low half not yet added into the high half) live in the high
//     lane, S and the pending exponent P in both;
//   * a rotated add (pw_combine) runs one add-with-carry chain per half: the low lane's carry
//     out is not propagated but handed to the high lane (one DPP swap) as its carry-in for the
//     NEXT combine (so the two halves never wait for each other); publishing folds it first;
//   * the inner product a b mod 2^N' + 1 (N' = 2 64 HL) is split by Karatsuba on the halves:
//     with X^2 = -1,  a b = a0b0 - a1b1 + X ((a0+a1)(b0+b1) - a0b0 - a1b1); the low lane
//     computes a0 b0 and the low columns of the middle product, the high lane a1 b1 and the
//     high columns, and each keeps / hands over (through LDS) the parts that land in its half.
// Exchange layout, pending exponents, weights, output and HBM format are those of k_pwss.
#pragma once
#include "pkernels.hpp"

// lanes 2i <-> 2i+1: one v_mov_b32_dpp quad_perm:[1,0,3,2]
__device__ __forceinline__ int p2_swap(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ u32 p2_swapu(u32 v) { return (u32)p2_swap((int)v); }
__device__ __forceinline__ u64 p2_swap64(u64 v) { return ((u64)p2_swapu((u32)(v >> 32)) << 32) | p2_swapu((u32)v); }

template <int HL>
__device__ __forceinline__ u32 p2_word(const u64 (&L)[HL], int k) { return (u32)(L[k >> 1] >> (32 * (k & 1))); }
template <int HL>
__device__ __forceinline__ void p2_setword(u64 (&L)[HL], int k, u32 v)
{
    if (k & 1) L[k >> 1] = (L[k >> 1] & 0xffffffffull) | ((u64)v << 32);
    else L[k >> 1] = (L[k >> 1] & ~0xffffffffull) | v;
}

// the high lane adds its pending carry C into its words (fast path: word 0 only, unless a lane
// of the wave overflows: probability ~2^-32); C = 0 after, T += the carry out
template <int HL>
__device__ __forceinline__ void p2_fold(u64 (&L)[HL], int &T, int &C, bool hi)
{
    const u32 w = (u32)L[0], n = w + (u32)(hi ? C : 0);
    if (!__any(hi && n < w)) {
        if (hi) L[0] = (L[0] & ~0xffffffffull) | n;
        C = 0;
        return;
    }
    if (hi) {
        u32 c = (u32)C;
#pragma unroll
        for (int k = 0; k < 2 * HL; ++k) p2_setword<HL>(L, k, __builtin_addc(p2_word<HL>(L, k), 0u, c, &c));
        T += (int)c;
    }
    C = 0;
}

// pw_norm for the split value: subtract D = T + 1 from the whole value so the top is -1
// (fast path: the low lane's word 0 absorbs D); T is meaningful in the high lane only
template <int HL>
__device__ __forceinline__ void p2_norm(u64 (&L)[HL], int &T, bool hi)
{
    const int To = p2_swap(T);
    const int D = (hi ? T : To) + 1;
    const u32 w0 = (u32)L[0], n0 = w0 - (u32)D;
    const bool spill = !hi && (D > 0 ? w0 < (u32)D : (D < 0 ? n0 < (u32)(-D) : false));
    if (!__any(spill)) {
        if (!hi) L[0] = (L[0] & ~0xffffffffull) | n0;
        else T = -1;
        return;
    }
    const u32 dh = D < 0 ? ~0u : 0u;
    u32 b = 0;
    if (!hi) {
#pragma unroll
        for (int k = 0; k < 2 * HL; ++k) p2_setword<HL>(L, k, __builtin_subc(p2_word<HL>(L, k), k == 0 ? (u32)D : dh, b, &b));
    }
    const int bl = p2_swap((int)b);
    if (hi) {
        b = (u32)bl;
#pragma unroll
        for (int k = 0; k < 2 * HL; ++k) p2_setword<HL>(L, k, __builtin_subc(p2_word<HL>(L, k), dh, b, &b));
        T = (D < 0) - (int)b - 1;
    }
}

// publish: exact words (fold), top -1 (norm), the lane's 2 HL words at rows hf 2HL + k,
// column t; the high lane writes the top + sign, the low lane the pending exponent
template <int M, int LK>
__device__ __forceinline__ void p2_publish(u64 (&L)[M / 2], int &T, int S, int &C, unsigned P, u32 *Xw, int *TT,
                                           unsigned *PP, int t, int hf)
{
    constexpr int K = 1 << LK, HL = M / 2;
    const bool hi = hf != 0;
    p2_fold<HL>(L, T, C, hi);
    p2_norm<HL>(L, T, hi);
    u32 *col = Xw + (size_t)(hf * 2 * HL) * K + t;
#pragma unroll
    for (int j = 0; j < HL; ++j) {
        col[(2 * j) * K] = (u32)L[j];
        col[(2 * j + 1) * K] = (u32)(L[j] >> 32);
    }
    if (hi) TT[t] = 2 * T + S;
    else PP[t] = P;
}

// r = alpha own + 2^E x_q (pw_combine, one half per lane).  Global output word g = hf M + k
// takes alignbit(w_g, w_(g-1)), w_i = the partner's word (i - Yw) mod 2M, complemented when
// wrapped (i < Yw) XOR negated.  Low lane: carry-in 1 (the rotation's +1), its carry out becomes
// the high lane's pending C; high lane: carry-in the old C, carry out into T.
template <int M, int LK>
__device__ __forceinline__ void p2_combine(u64 (&L)[M / 2], int &T, int &S, int &C, int alpha, const u32 *Xw,
                                           const int *TT, int q, unsigned E, int hf)
{
    constexpr int K = 1 << LK, NW = 2 * M, HW = M, HL = M / 2;
    constexpr unsigned NP = 64 * M;
    const bool hi = hf != 0;
    const int packed = TT[q], Tq = packed >> 1, Sq = packed & 1;
    bool neg = E >= NP;
    if (neg) E -= NP;
    const int Yw = ((int)E - 1) >> 5;                    // E = 0: Yw = -1, s5 = 32
    const unsigned sh = (unsigned)(32 * (Yw + 1)) - E;   // 32 - s5, in [0, 31]
    if (alpha == 0) {
#pragma unroll
        for (int j = 0; j < HL; ++j) L[j] = 0;
        T = 0;
        S = 0;
        C = 0;
    } else if (alpha < 0) {
        S ^= 1;
    }
    neg ^= (S ^ Sq) != 0;
    const u32 smask = neg ? ~0u : 0u;
    const int g0 = hf * HW;                              // first global output word of this lane
    // source of global word g0 - 1 + j at b0[j K] (not wrapped) or bw0[j K] (wrapped: g < Yw)
    const u32 *b0 = Xw + q + (g0 - 1 - Yw) * K;
    const u32 *bw0 = b0 + NW * K;
    const int yl = Yw - g0 + 1;                          // j < yl: wrapped
    u32 wv[HW + 1];
#pragma unroll
    for (int j = 0; j <= HW; ++j) {
        const bool wr = j < yl;
        wv[j] = (wr ? bw0 : b0)[j * K] ^ (wr ? ~smask : smask);
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
    u32 c = hi ? (u32)C : 1u;
#pragma unroll
    for (int k = 0; k < HW; ++k) {
        const u32 o = __builtin_amdgcn_alignbit(wv[k + 1], wv[k], sh);
        p2_setword<HL>(L, k, __builtin_addc(p2_word<HL>(L, k), o, c, &c));
    }
    const int cout = (int)c, other = p2_swap(cout);
    if (hi) {
        T += cout;
        C = other;   // the low lane's carry out, into the next combine (or fold)
    }
    if (__any(Tq != -1)) {   // rare: add cv 2^E', cv = -(1 + T_q) (negated when E >= N')
        // exact words first (no pending carry), then one chain over both halves
        if (hi) {
            u32 f = (u32)C;
#pragma unroll
            for (int k = 0; k < HW; ++k) p2_setword<HL>(L, k, __builtin_addc(p2_word<HL>(L, k), 0u, f, &f));
            T += (int)f;
        }
        C = 0;
        const int cv = neg ? 1 + Tq : -1 - Tq;
        const i64 d = (i64)cv * ((i64)1 << (32 - sh));
        const u32 dl = (u32)d, dhi = (u32)((u64)d >> 32), sx = d < 0 ? ~0u : 0u;
        u32 cc = 0;
        if (!hi) {
#pragma unroll
            for (int k = 0; k < HW; ++k) {
                const u32 ad = k < Yw ? 0u : k == Yw ? dl : k == Yw + 1 ? dhi : sx;
                p2_setword<HL>(L, k, __builtin_addc(p2_word<HL>(L, k), ad, cc, &cc));
            }
        }
        const int ccl = p2_swap((int)cc);
        if (hi) {
            cc = (u32)ccl;
#pragma unroll
            for (int k = 0; k < HW; ++k) {
                const int g = HW + k;
                const u32 ad = g < Yw ? 0u : g == Yw ? dl : g == Yw + 1 ? dhi : sx;
                p2_setword<HL>(L, k, __builtin_addc(p2_word<HL>(L, k), ad, cc, &cc));
            }
            T += (int)cc + (Yw == NW - 1 ? (int)(d >> 32) : (d < 0 ? -1 : 0));
        }
    }
}

// one forward (DIF) or inverse (DIT) length-K transform (pw_transform) on the split values:
// partners share a wave when h < 32 (32 pieces per wave)
template <int M, int LK, int DIR>
__device__ __forceinline__ void p2_transform(u64 (&L)[M / 2], int &T, int &S, int &C, unsigned &P, u32 *Xw, int *TT,
                                             unsigned *PP, unsigned TH, int t, int hf)
{
    constexpr int K = 1 << LK, lk = LK;
    constexpr unsigned N2 = 128 * M;
    for (int jj = 0; jj < lk; ++jj) {
        const int j = DIR == 0 ? jj : lk - 1 - jj;
        const int h = K >> (j + 1);
        const int q = t ^ h;
        const bool top = !(t & h);
        const int qt = t & ~h;
        const unsigned tw = (unsigned)((qt & (h - 1)) << j) * (2 * TH);
        const bool cross = h >= 32;
        p2_publish<M, LK>(L, T, S, C, P, Xw, TT, PP, t, hf);
        if (cross) __syncthreads(); else pw_wave_sync();
        const unsigned Pq = PP[q];
        unsigned E;
        if (DIR == 0) {
            E = pw_mod(Pq + N2 - P, N2);
            p2_combine<M, LK>(L, T, S, C, top ? 1 : -1, Xw, TT, q, E, hf);
            if (!top) P = pw_mod(P + tw, N2);
        } else {
            E = top ? pw_mod(Pq + 2 * N2 - tw - P, N2) : pw_mod(Pq + N2 - P + tw, N2);
            p2_combine<M, LK>(L, T, S, C, top ? 1 : -1, Xw, TT, q, E, hf);
            if (!top) P = pw_mod(P + N2 - tw, N2);
        }
        if (cross) __syncthreads(); else pw_wave_sync();
    }
}

// canonical residue (pw_canon) of the split value: limbs in [0, 2^N'), returns 1 (both lanes)
// for 2^N' (limbs 0).  Chains run low lane, then high lane (DPP-handed carries).
template <int HL>
__device__ __forceinline__ int p2_canon(u64 (&L)[HL], int &T, int &C, bool hi)
{
    p2_fold<HL>(L, T, C, hi);
    const int To = p2_swap(T);
    const int Tall = hi ? T : To;
    i128 acc = 0;
    int c0 = 0;
    if (!hi) {   // L - T over the low half
        acc = -(i128)Tall;
#pragma unroll
        for (int j = 0; j < HL; ++j) {
            acc += (i128)L[j];
            L[j] = (u64)acc;
            acc >>= 64;
        }
        c0 = (int)(i64)acc;
    }
    const int c0h = p2_swap(c0);
    int c1 = 0;
    if (hi) {
        acc = (i128)c0h;
#pragma unroll
        for (int j = 0; j < HL; ++j) {
            acc += (i128)L[j];
            L[j] = (u64)acc;
            acc >>= 64;
        }
        c1 = (int)(i64)acc;   // value == L - c1 now
    }
    const int c1o = p2_swap(c1);
    const int c1all = hi ? c1 : c1o;
    int c2 = 0;
    if (!hi) {
        acc = -(i128)c1all;
#pragma unroll
        for (int j = 0; j < HL; ++j) {
            acc += (i128)L[j];
            L[j] = (u64)acc;
            acc >>= 64;
        }
        c2 = (int)(i64)acc;
    }
    const int c2h = p2_swap(c2);
    int z = 0;
    if (hi) {
        acc = (i128)c2h;
#pragma unroll
        for (int j = 0; j < HL; ++j) {
            acc += (i128)L[j];
            L[j] = (u64)acc;
            acc >>= 64;
        }
        z = (i64)acc != 0;    // the second fold wrapped: the value is 2^N' == -1
    }
    const int zo = p2_swap(z);
    const int zall = hi ? z : zo;
    if (zall) {
#pragma unroll
        for (int j = 0; j < HL; ++j) L[j] = 0;
    }
    T = 0;
    return zall;
}

// Stream the columns of a digit product into 64-bit limbs (the product scan of pw_mulmod):
// column c (value < 2^63) sits at bit OFF + 28 c; limb k (bits 64 k ..) is handed to emit(k, v)
// in increasing k, k < KMAX.  Columns c in [C0, C1] of  sum_i a_i b_(c - i), i in [I0(c), I1(c)].
template <int ND, int C0, int C1, int OFF, int KMAX, typename Emit>
__device__ __forceinline__ void p2_columns(const u32 (&a)[ND], const u32 (&b)[ND], Emit &&emit)
{
    constexpr int DB = 28;
    u128 acc = 0;
    int pos = 0, k = 0;   // compile-time after unrolling: acc holds bits [pos, ...)
#pragma clang loop unroll(full)
    for (int c = C0; c <= C1; ++c) {
        u64 col = 0;
        const int i0 = c < ND ? 0 : c - ND + 1, i1 = c < ND ? c : ND - 1;
#pragma clang loop unroll(full)
        for (int i = i0; i <= i1; ++i) col += (u64)a[i] * b[c - i];
        __builtin_amdgcn_sched_barrier(0);   // one column's products live at a time (VGPRs)
        const int bitpos = OFF + DB * c;
        acc += (u128)col << (bitpos - pos);
        const bool last = c == C1;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            if (k < KMAX && (last || bitpos + DB - pos >= 64)) {
                emit(k, (u64)acc);
                acc >>= 64;
                pos += 64;
                ++k;
            }
        }
    }
    // flush (a product's value fits KMAX limbs: nothing is left in acc)
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        if (k < KMAX) {
            emit(k, (u64)acc);
            acc >>= 64;
            ++k;
        }
    }
}

// z = a b mod 2^N' + 1 for canonical split values a0 | a1, b0 | b1 (below 2^N': an operand
// equal to 2^N' == -1 is passed as 1 with the product's sign flipped, by the caller):
// low lane  keeps S0 - R = P0L + P0H - (the part of its middle columns above X),
//           hands over D0 + PmL = P0H - P0L + (its middle columns below X);
// high lane keeps -(S2 + Q_top) = -(P2L + P2H) - (middle columns above X^2),
//           hands over D2 - Q_low = P2H - P2L - (its middle columns between X and X^2);
// so  z_lo = P0L + P0H + P2H - P2L - PmH,  z_hi = P0H - P0L - P2L - P2H + PmL - PmT.
// XE: the LDS word rows (publish layout); CE: 2K ints.  Result: Z (the lane's half), T (high
// lane), no pending carry.
template <int M, int LK>
__device__ __forceinline__ void p2_mulmod(u64 (&Z)[M / 2], int &T, const u64 (&La)[M / 2], const u64 (&Lb)[M / 2],
                                          u32 *XE, int *CE, int t, int hf)
{
    constexpr int K = 1 << LK, HL = M / 2, DB = 28, ND = (64 * HL + DB - 1) / DB;
    static_assert(ND <= 32, "middle-product columns must stay below 2^63");
    const bool hi = hf != 0;
    u32 ad[ND], bd[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const int b0 = d * DB, li = b0 >> 6, sh = b0 & 63;
        u64 x = La[li] >> sh, y = Lb[li] >> sh;
        if (sh + DB > 64 && li + 1 < HL) {
            x |= La[li + 1] << (64 - sh);
            y |= Lb[li + 1] << (64 - sh);
        }
        ad[d] = (u32)(x & ((1u << DB) - 1));
        bd[d] = (u32)(y & ((1u << DB) - 1));
    }
    // (A) own half product P = P_L + P_H X: S = P_L + P_H into Z, D = P_H - P_L straight into
    // this lane's exchange rows (the publish layout: 32-bit word rows of column t only -- other
    // waves may still be exchanging in their own columns; keeping D out of VGPRs is what holds
    // the kernel to 4 waves per SIMD)
    u32 *mine = XE + (size_t)(hf * 2 * HL) * K + t, *theirs = XE + (size_t)((1 - hf) * 2 * HL) * K + t;
    u32 cs = 0, bw = 0;   // carry of S, borrow of D (both weigh X)
    p2_columns<ND, 0, 2 * ND - 2, 0, 2 * HL>(ad, bd, [&](int k, u64 v) {
        if (k < HL) {
            Z[k] = v;
        } else {
            const int j = k - HL;
            const u64 pl = Z[j];
            u32 c1;
            const u32 s0 = __builtin_addc((u32)pl, (u32)v, cs, &c1);
            const u32 s1 = __builtin_addc((u32)(pl >> 32), (u32)(v >> 32), c1, &cs);
            u32 b1;
            mine[(size_t)(2 * j) * K] = __builtin_subc((u32)v, (u32)pl, bw, &b1);
            mine[(size_t)(2 * j + 1) * K] = __builtin_subc((u32)(v >> 32), (u32)(pl >> 32), b1, &bw);
            Z[j] = ((u64)s1 << 32) | s0;
        }
    });
    // (B) middle-product digits: the sums of both halves' digits (< 2^29), identical in both lanes
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        ad[d] += p2_swapu(ad[d]);
        bd[d] += p2_swapu(bd[d]);
    }
    // Zk: value kept in Z (S form) with its carry zc (weighs X); Dv: value handed over, carry dc
    int zc = (int)cs, dc = -(int)bw;
    if (!hi) {
        // columns [0, ND): bits [0, 28 ND + ..): limbs < HL add into D (PmL), limbs >= HL
        // subtract from S at k - HL (R, the part above X)
        u32 ca = 0, cr = 0;
        p2_columns<ND, 0, ND - 1, 0, HL + 2>(ad, bd, [&](int k, u64 v) {
            if (k < HL) {
                u32 c1;
                u32 *w = mine + (size_t)(2 * k) * K;
                w[0] = __builtin_addc(w[0], (u32)v, ca, &c1);
                w[K] = __builtin_addc(w[K], (u32)(v >> 32), c1, &ca);
            } else {
                const int j = k - HL;
                u32 b1;
                const u32 x0 = __builtin_subc((u32)Z[j], (u32)v, cr, &b1);
                const u32 x1 = __builtin_subc((u32)(Z[j] >> 32), (u32)(v >> 32), b1, &cr);
                Z[j] = ((u64)x1 << 32) | x0;
            }
        });
        // the R borrow keeps rippling through S's remaining limbs
#pragma unroll
        for (int j = 2; j < HL; ++j) {
            u32 b1;
            const u32 x0 = __builtin_subc((u32)Z[j], 0u, cr, &b1);
            const u32 x1 = __builtin_subc((u32)(Z[j] >> 32), 0u, b1, &cr);
            Z[j] = ((u64)x1 << 32) | x0;
        }
        zc -= (int)cr;
        dc += (int)ca;
    } else {
        // columns [ND, 2 ND - 2): bit 28 c - 64 HL relative to X (>= 0); limbs < HL subtract
        // from D (Q_low), limbs >= HL add into S (Q_top, kept negated below)
        u32 bq = 0, ct = 0;
        p2_columns<ND, ND, 2 * ND - 2, -64 * HL, HL + 1>(ad, bd, [&](int k, u64 v) {
            if (k < HL) {
                u32 b1;
                u32 *w = mine + (size_t)(2 * k) * K;
                w[0] = __builtin_subc(w[0], (u32)v, bq, &b1);
                w[K] = __builtin_subc(w[K], (u32)(v >> 32), b1, &bq);
            } else {
                const int j = k - HL;
                u32 c1;
                const u32 x0 = __builtin_addc((u32)Z[j], (u32)v, ct, &c1);
                const u32 x1 = __builtin_addc((u32)(Z[j] >> 32), (u32)(v >> 32), c1, &ct);
                Z[j] = ((u64)x1 << 32) | x0;
            }
        });
#pragma unroll
        for (int j = 1; j < HL; ++j) {
            u32 c1;
            const u32 x0 = __builtin_addc((u32)Z[j], 0u, ct, &c1);
            const u32 x1 = __builtin_addc((u32)(Z[j] >> 32), 0u, c1, &ct);
            Z[j] = ((u64)x1 << 32) | x0;
        }
        zc += (int)ct;
        dc -= (int)bq;
    }
    // (C) hand D over: the rows are written, the carries follow
    CE[2 * t + hf] = dc;
    pw_wave_sync();   // the pair shares a wave
    const int oc = CE[2 * t + (1 - hf)];
    // low lane: z_lo = Z + D_hi; high lane: z_hi = D_lo - Z
    i128 acc = 0;
#pragma unroll
    for (int j = 0; j < HL; ++j) {
        const u64 o = (u64)theirs[(size_t)(2 * j) * K] | ((u64)theirs[(size_t)(2 * j + 1) * K] << 32);
        acc += hi ? (i128)o - (i128)Z[j] : (i128)Z[j] + (i128)o;
        Z[j] = (u64)acc;
        acc >>= 64;
    }
    const int ztop = (int)(i64)acc + (hi ? oc - zc : zc + oc);   // weighs X (low) or X^2 (high)
    pw_wave_sync();   // the exchange rows are read before anything reuses them
    // the low half's overflow moves into the high half; the high half's is the top
    const int zl = p2_swap(ztop);
    if (hi) {
        acc = (i128)zl;
#pragma unroll
        for (int j = 0; j < HL; ++j) {
            acc += (i128)Z[j];
            Z[j] = (u64)acc;
            acc >>= 64;
        }
        T = ztop + (int)(i64)acc;
    } else {
        T = 0;
    }
}

// k_pw2<M, LK, FUSE>: k_pwss with two threads per piece (2K threads per slot); same arguments,
// inputs and outputs.
template <int M, int LK, int FUSE>
__global__ __launch_bounds__(2 << LK) __attribute__((amdgpu_waves_per_eu(4))) void k_pw2(u64 *digA, u64 *cbA, int *topA, const u64 *digB, const u64 *cbB,
                                                 const int *topB, int l, u64 *digC, u64 *cbC, int *topC,
                                                 unsigned long long *dbg)
{
    (void)dbg;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int K = 1 << LK, HL = M / 2, lk = LK;
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    const int tau = threadIdx.x, t = tau >> 1, hf = tau & 1;
    const bool hi = hf != 0;
    u64 *X = (u64 *)smem;                        // (M + 1) K limbs (2M + 2 word rows in the transforms)
    u32 *Xw = (u32 *)smem;
    int *TT = (int *)(X + (size_t)(M + 1) * K);  // K
    unsigned *PP = (unsigned *)(TT + K);         // K
    int *H = (int *)(PP + K);                    // l
    int *CE = H + l;                             // 2K
    const int cbw = cb_words(l);
    constexpr int CLP = pw_piece_limbs<M, LK>();
    static_assert(HL >= CLP + 1, "a loaded piece (+ its carry limb) must fit the low half");
    // load: the low lane the piece of A, the high lane the piece of B (each a full piece value
    // in HL limbs, top -1 / 0), then the low lane takes B's piece and both tops go high
    u64 Lx[HL];
    int Tx;
    long slot = blockIdx.x;
    if (FUSE == 0) {
        if (!hi) pw_load_piece<HL, CLP>(Lx, Tx, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA[slot], l, t);
        else pw_load_piece<HL, CLP>(Lx, Tx, digB + (size_t)slot * l, cbB + (size_t)slot * cbw, topB[slot], l, t);
        __syncthreads();   // every piece read before any output limb is written (in place on A)
    } else {
        const long b = blockIdx.x, nb = gridDim.x, main = nb - nb % 16;   // XCD-aware pair order (k_pwss)
        if (b < main) {
            const long x = b & 7, j = b >> 3;
            slot = 2 * (((j >> 1) << 3) + x) + (j & 1);
        }
        if (!hi) pw_load_pair_bfly<HL, CLP>(Lx, Tx, digA, cbA, topA, slot & ~1L, l, cbw, t, slot & 1);
        else pw_load_pair_bfly<HL, CLP>(Lx, Tx, digB, cbB, topB, slot & ~1L, l, cbw, t, slot & 1);
    }
    const int To = p2_swap(Tx);
    u64 La[HL], Lb[HL];
    int Ta, Tb;
#pragma unroll
    for (int j = 0; j < HL; ++j) {
        const u64 y = p2_swap64(Lx[j]);
        La[j] = hi ? (To ? ~0ull : 0ull) : Lx[j];
        Lb[j] = hi ? (Tx ? ~0ull : 0ull) : y;
    }
    Ta = hi ? To : 0;
    Tb = hi ? Tx : 0;
    // transforms of both operands, product, inverse, un-weighting (pw_slot_product)
    const unsigned TH = NP >> lk;
    int Sa = 0, Sb = 0, Ca = 0, Cb = 0;
    unsigned Pa = (unsigned)t * TH, Pb = Pa;
    p2_transform<M, LK, 0>(La, Ta, Sa, Ca, Pa, Xw, TT, PP, TH, t, hf);
    p2_transform<M, LK, 0>(Lb, Tb, Sb, Cb, Pb, Xw, TT, PP, TH, t, hf);
    const int ca = p2_canon<HL>(La, Ta, Ca, hi), cb = p2_canon<HL>(Lb, Tb, Cb, hi);
    u64 Z[HL];
    int Tz, Sz = Sa ^ Sb ^ ca ^ cb, Cz = 0;
    // an operand equal to 2^N' == -1 (limbs 0, flag set) enters the product as 1 with the
    // sign flipped: (-1) b = -(1 b)  (cf. the flag c of mul_fft.c:3250)
    if (ca && !hi) La[0] = 1;
    if (cb && !hi) Lb[0] = 1;
    p2_mulmod<M, LK>(Z, Tz, La, Lb, Xw, CE, t, hf);
    unsigned Pz = pw_mod(Pa + Pb, N2);
    p2_transform<M, LK, 1>(Z, Tz, Sz, Cz, Pz, Xw, TT, PP, TH, t, hf);
    {
        const unsigned un = (unsigned)t * TH + lk;
        const unsigned F = pw_mod(Pz + N2 - un, N2);
        p2_publish<M, LK>(Z, Tz, Sz, Cz, Pz, Xw, TT, PP, t, hf);
        pw_wave_sync();                                   // own column only
        p2_combine<M, LK>(Z, Tz, Sz, Cz, 0, Xw, TT, t, F, hf);
        __syncthreads();                                  // the u64 rows below cross columns
    }
    const int zt = p2_canon<HL>(Z, Tz, Cz, hi);
    const int topbit = (int)(Z[HL - 1] >> 63);
    const int tbo = p2_swap(topbit);
    const int neg = zt || (hi ? topbit : tbo);
#pragma unroll
    for (int j = 0; j < HL; ++j) X[(size_t)(hf * HL + j) * K + t] = Z[j];
    if (hi) {
        X[(size_t)M * K + t] = (u64)zt;
        TT[t] = neg;
    }
    __syncthreads();
    if (FUSE == 0)
        pw_slot_output<M, LK, 2 * K>(X, TT, H, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA + slot, l, tau);
    else
        pw_slot_output<M, LK, 2 * K>(X, TT, H, digC + (size_t)slot * l, cbC + (size_t)slot * cbw, topC + slot, l, tau);
}

// LDS of one k_pw2 workgroup: k_pwss's plus the product exchange carries
__host__ __device__ constexpr size_t pw2_lds_bytes(int M, int K, int l) { return pw_lds_bytes(M, K, l) + (size_t)8 * K; }
