// pkernels.hpp -- sub-quadratic pointwise products mod p = 2^N + 1 for big coefficients
// (the nested negacyclic transform of FFT_mulmod_2expp1 /
// fft_mulmod_2expp1, mul_fft.c:2998-3167, FFT/IFFT_radix2_negacyclic :1290, :1861).
//
// One workgroup computes one product a b mod p (a, b in the reduced HBM form, N = 64 l bits):
//   * a, b are cut into K = 2^lk pieces of B = N/K bits (thread t owns piece t);
//   * the negacyclic convolution of the pieces (X^K == -1 with X = 2^B, so it IS the
//     product mod p) is computed in the inner ring R' = Z/(2^N' + 1), N' = 64 M, with
//     N' >= 2B + lk + 4 so every signed convolution coefficient |c_t| < K 2^(2B+2) is
//     recovered exactly from its residue (the reference instead restores the top
//     with a naive convolution of the low limbs, :3088; headroom is cheaper here);
//   * negacyclic weights theta^t, theta = 2^(N'/K) a 2K-th root of unity, then a length-K
//     cyclic DIF transform with root omega = theta^2 = 2^(2N'/K), pointwise products in R',
//     DIT inverse, division by K and un-weighting.  Only omega must be a power of two:
//     N' is a multiple of K/2 (not K), and when N'/K is a half-integer the odd weights use
//     sqrt(2) = 2^(N'/4) (2^(N'/2) - 1) in R' (pw_sqrt2, one in-thread half swap) -- the
//     identity of the reference's FFT_radix2_butterfly_sqrt2 (mul_fft.c:580-640) applied to the inner
//     ring.  That lets N' be the smallest multiple of 64 K/2 bits above the headroom bound
//     (C3: 1152 instead of 1280 bits, C4: 1280 instead of 1536).
//   All the other multiplications are by powers of two.
// Thread t holds its coefficient (M limbs + a small signed top word, value =
// limbs + top 2^N') in registers: additions are in-thread carry chains
// (v_add_co / v_addc).  A butterfly partner is read from LDS (limb-major,
// conflict-free) already rotated by the relative exponent; each thread keeps a
// *pending* exponent so its own value is never rotated.  The inner products are
// in-thread product-scanning schoolbook on 32-bit digits (v_mad_u64_u32).
// The coefficients are then summed (with their signs and the negacyclic wrap) into
// the l output limbs and stored in the reduced HBM form the inverse pass loads.
#pragma once
#include <type_traits>
#include "coeff.hpp"

// LDS of one k_pwss workgroup: M K limbs (the exchange rows, then the coefficients; the l
// output overflows alias them) + tops + pending exponents.  C3 (M = 18, K = 256): 38 912 B,
// so four workgroups share a CU's 160 KiB (pw_wpe).
// Tight form (PW_TIGHT9, K = 512): no top / pending-exponent arrays beside the exchange rows --
// a level's partner tops and exponents go by a wave shuffle (partner in the wave) or through
// the first two exchange rows before the words are published (two more barriers), and the
// signed coefficients are stored as two's complement (no sign array) -- so the workgroup needs
// exactly M K 8 bytes: 80 KiB at C4 (M = 20), two workgroups per CU instead of one.
#ifndef PW_TIGHT9
#define PW_TIGHT9 1   // 0: the round-3 form (86 KB, one workgroup per CU at C4), for A/B builds
#endif
__host__ __device__ constexpr bool pw_tight(int K) { return PW_TIGHT9 && K == 512; }
// operand B's pieces loaded after A's forward transform (pw_slot_product's loadB): the tight
// form only (C4 pointwise 39.0 -> 37.7 ms; at l = 2048, four workgroups per CU, 0.5-2 % slower:
// profiles/r04/pw_tight_ab.txt)
#ifndef PW_LATE_B_ALL
#define PW_LATE_B_ALL 0   // A/B builds: the late operand-B load at every size
#endif
__host__ __device__ constexpr bool pw_late_b(int K) { return pw_tight(K) || PW_LATE_B_ALL; }
// inputs in flight in the late operand-B quad loader: one (A's transformed limbs are live; with two
// the C4 kernel spilled 40 B per lane, with one it has no scratch at all, at equal speed:
// C4 pointwise 32.41 vs 32.49 ms, profiles/r05/pw_late_infl_ab.txt).  A/B builds: -DPW_LATE_INFL=2
#ifndef PW_LATE_INFL
#define PW_LATE_INFL 1
#endif
#ifndef PW_A_INFL
#define PW_A_INFL 2       // A/B builds: inputs in flight in operand A's quad loader (1, 2 or 4)
#endif
#ifndef PW_QUAD4
#define PW_QUAD4 0        // A/B builds: the quad loader's four inputs in flight at once
#endif

__host__ __device__ constexpr size_t pw_lds_bytes(int M, int K, int l)
{
    return ((size_t)M * K * 8 > (size_t)l * 4 ? (size_t)M * K * 8 : (size_t)l * 4) + (pw_tight(K) ? 0 : (size_t)K * 8);
}

// waves per SIMD k_pwss is compiled for: 4 (VGPRs <= 128) where the LDS fits 1024 threads per
// CU (K = 256: four workgroups; the tight K = 512 form: two), else 2 (the compiler's choice,
// ~140-170 VGPRs)
template <int M, int LK>
__host__ __device__ constexpr int pw_wpe()
{
    return pw_lds_bytes(M, 1 << LK, 64 * M) * (1024 >> LK) <= 160 * 1024 ? 4 : 2;
}
// partner-word prefetch distance of pw_combine for that budget
#ifndef PW_PD_TIGHT
#define PW_PD_TIGHT 16
#endif
template <int M, int LK>
#ifndef PW_PD_WIDE
#define PW_PD_WIDE 16     // A/B builds: the same for the K = 256 kernels
#endif
__host__ __device__ constexpr int pw_pd() { return pw_wpe<M, LK>() == 4 ? (pw_tight(1 << LK) ? PW_PD_TIGHT : PW_PD_WIDE) : 2 * M; }

// Exchange format: thread t publishes its value as 2M 32-bit words, word k at
// Xw[k K + t] (conflict-free for any rotation), top in TT[t].  Before publishing,
// pw_norm moves the top to -1 (almost always exactly): the reader's rotation then
// needs no correction term, only a complement mask and one carry chain.

// L + T 2^N' == (L - (T + 1)) - 2^N'  (mod p'): subtract D = T + 1; returns the new top
// (-1 unless the subtraction left [0, 2^N'), which needs L < D or L - D >= 2^N').
// PW_NORM_SPILL_ALL (test builds only, libmpfft_pwspill.so): every lane takes the device form's
// rare branch below -- keeps its top -- so the readers' T_q != -1 path runs on every exchange
// (tests/test_gpu_parity.py::test_pointwise_norm_spill_branch)
#ifndef PW_NORM_SPILL_ALL
#define PW_NORM_SPILL_ALL 0
#endif
template <int M>
__host__ __device__ __forceinline__ int pw_norm(u64 (&L)[M], int T)
{
    const int D = T + 1;
#if defined(__HIP_DEVICE_COMPILE__)
    // Device form (the kernel is VALU-bound): a small D only moves the low word unless it
    // under/overflows (probability ~2^-32 per lane); such a lane keeps its top, which every
    // reader handles (pw_combine's Tq != -1 branch) -- no full chain, whose rewrite of all M
    // limbs under a branch made the compiler keep a second copy of L live across the levels'
    // loop and spill it there (C4 pointwise 34.9 -> 34.1 ms, C3 3.47 -> 3.43 ms)
    {
        const u32 w0 = (u32)L[0], n0 = w0 - (u32)D;
        const bool spill = PW_NORM_SPILL_ALL || (D > 0 ? w0 < (u32)D : (D < 0 ? n0 < (u32)(-D) : false));
        L[0] = (L[0] & ~0xffffffffull) | (spill ? w0 : n0);
        return spill ? T : -1;
    }
#endif
    const u32 dh = D < 0 ? ~0u : 0u;
    u32 b = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const u32 lo = __builtin_subc((u32)L[j], j == 0 ? (u32)D : dh, b, &b);
        const u32 hi = __builtin_subc((u32)(L[j] >> 32), dh, b, &b);
        L[j] = ((u64)hi << 32) | lo;
    }
    // L - D = L' + ((D < 0) - b) 2^N'
    return (D < 0) - (int)b - 1;
}

// Values are kept with a sign flag S: the represented value is (-1)^S (L + T 2^N'), so
// a butterfly's "-own" is a flag flip and every combine is own + (+-) rotated partner,
// the partner's sign folded into the complement mask.
// r = alpha * own + 2^E * x_q  (mod p', not reduced); alpha in {-1, 0, 1}.
// x_q: words Xw[k K + q], TT[q] = 2 T_q + S_q.  With E' = E mod N' = 32 Yw + s5, s5 in [1, 32]:
//   out = the N'-bit circular rotation of x_q's limbs by E', its low E' (wrapped) bits
//         complemented:  out_k = alignbit(w_k, w_(k-1), 32 - s5),
//         w_i = Xw[(i - Yw) mod 2M], complemented when i < Yw (i in [-1, 2M));
//   2^E' x_q == out + 1 - (1 + T_q) 2^E'   (rotation wraps negated; T_q 2^N' == -T_q);
//   negated (E >= N', or the signs differ):  ~out + 1 + (1 + T_q) 2^E'.
// After pw_norm T_q = -1 on all but ~2^-32 of the lanes (a lane whose low word would under- or
// overflow keeps its top, pw_norm's device form), so the (1 + T_q) term is a rare branch, and the
// whole sum is one add-with-carry chain with carry-in 1.
// packed: the partner's 2 T_q + S_q (TT[q], or a register in the tight form)
// FIXE >= 0: the caller guarantees E mod N' == FIXE, so the rotation is a compile-time constant
// and every wrap test, word address and complement mask below folds away (the forward
// transforms' first level, where E is exactly N'/2 for every thread: pw_transform)
template <int M, int LK, int PD = 2 * M, int FIXE = -1>
__host__ __device__ __forceinline__ void pw_combine(u64 (&L)[M], int &T, int &S, int alpha, const u32 *Xw,
                                                   int packed, int q, unsigned E)
{
    constexpr int K = 1 << LK, NW = 2 * M;
    constexpr unsigned NP = 64 * M;
    const int Tq = packed >> 1, Sq = packed & 1;
    bool neg = E >= NP;
    if (neg) E -= NP;
    if (FIXE >= 0) E = (unsigned)FIXE;
    const int Yw = ((int)E - 1) >> 5;                    // E = 0: Yw = -1, s5 = 32
    const unsigned sh = (unsigned)(32 * (Yw + 1)) - E;   // 32 - s5, in [0, 31]
    if (alpha == 0) {
#pragma unroll
        for (int j = 0; j < M; ++j) L[j] = 0;
        T = 0;
        S = 0;
    } else if (alpha < 0) {
        S ^= 1;
    }
    neg ^= (S ^ Sq) != 0;
    const u32 smask = neg ? ~0u : 0u;
    const u32 *bn = Xw + q - Yw * K;          // source word i >= Yw: bn[i K]
    const u32 *bw = bn + NW * K;              // i < Yw: wrapped
    // w_(-1): wrapped unless Yw = -1 (then it is word 0 and the funnel shift is 0).
    // Yw = -1 also reads row 2M at k = 2M - 1 (unused by the funnel): the buffer has it.
    u32 wprev = (-1 < Yw ? bw : bn)[-K] ^ (-1 < Yw ? ~smask : smask);
    u32 c = 1;
    // partner words are read PD ahead of their use: all NW at once by default (one or two
    // at a time, the compiler's own order, exposed the LDS latency per word); a bounded
    // distance where the kernel must fit 128 VGPRs (pw_wpe: more waves hide the latency)
    constexpr int D0 = PD < NW ? PD : NW;
    u32 wv[NW];
#pragma unroll
    for (int k = 0; k < D0; ++k) {
        const bool wr = k < Yw;
        wv[k] = (wr ? bw : bn)[k * K];
#if defined(__HIP_DEVICE_COMPILE__)
        if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
#endif
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        if (k + D0 < NW) {
            const bool wr2 = k + D0 < Yw;
            wv[k + D0] = (wr2 ? bw : bn)[(k + D0) * K];
        }
        const bool wr = k < Yw;
        const u32 w = wv[k] ^ (wr ? ~smask : smask);
#if defined(__HIP_DEVICE_COMPILE__)
        const u32 o = __builtin_amdgcn_alignbit(w, wprev, sh);
#else
        const u32 o = (u32)((((u64)w << 32) | wprev) >> sh);
#endif
        wprev = w;
        const u32 lw = (u32)(L[k >> 1] >> (32 * (k & 1)));
        const u32 r = __builtin_addc(lw, o, c, &c);
        if (k & 1) L[k >> 1] = (L[k >> 1] & 0xffffffffull) | ((u64)r << 32);
        else L[k >> 1] = (L[k >> 1] & ~0xffffffffull) | r;
#if defined(__HIP_DEVICE_COMPILE__)
        if (D0 < NW && (k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
#endif
    }
    T += (int)c;
    if (Tq != -1) {   // rare: add cv 2^E', cv = -(1 + T_q) (negated when E >= N')
        const int cv = neg ? 1 + Tq : -1 - Tq;
        const i64 d = (i64)cv * ((i64)1 << (32 - sh));
        const u32 dl = (u32)d, dhi = (u32)((u64)d >> 32), sx = d < 0 ? ~0u : 0u;
        u32 cc = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const u32 ad = k < Yw ? 0u : k == Yw ? dl : k == Yw + 1 ? dhi : sx;
            const u32 lw = (u32)(L[k >> 1] >> (32 * (k & 1)));
            const u32 r = __builtin_addc(lw, ad, cc, &cc);
            if (k & 1) L[k >> 1] = (L[k >> 1] & 0xffffffffull) | ((u64)r << 32);
            else L[k >> 1] = (L[k >> 1] & ~0xffffffffull) | r;
        }
        T += (int)cc + (Yw == NW - 1 ? (int)(d >> 32) : (d < 0 ? -1 : 0));
    }
}

// canonical residue of L + T 2^N' (== L - T): limbs in [0, 2^N'), returns 1 for 2^N' (L = 0)
template <int M>
__host__ __device__ __forceinline__ int pw_canon(u64 (&L)[M], int T)
{
    i128 acc = -(i128)T;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        acc += (i128)L[j];
        L[j] = (u64)acc;
        acc >>= 64;
    }
    const int c1 = (int)(i64)acc;   // value == L - c1 now, |c1| <= 1
    acc = -(i128)c1;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        acc += (i128)L[j];
        L[j] = (u64)acc;
        acc >>= 64;
    }
    if ((i64)acc != 0) {   // the second fold wrapped: the value is 2^N' == -1
#pragma unroll
        for (int j = 0; j < M; ++j) L[j] = 0;
        return 1;
    }
    return 0;
}

// L + T 2^N'  <-  (2^(N'/2) - 1) (L + T 2^N')  mod p'  (M even; lo, hi = the low and high
// M/2 limbs of L):  2^(N'/2) (lo + hi 2^(N'/2) + T 2^N') == lo 2^(N'/2) - hi - T 2^(N'/2), so
// the product is (T - hi - lo) + (lo - hi - T) 2^(N'/2): two interleaved chains, then the low
// chain's carry (in [-2, 1]) rippled into the high half.  The new top is small (|T'| <= |T| + 3).
template <int M>
__host__ __device__ __forceinline__ void pw_sqrt2(u64 (&L)[M], int &T)
{
    static_assert(M % 2 == 0, "the half swap needs an even limb count");
    constexpr int H = M / 2;
    i128 a0 = (i128)T, a1 = -(i128)T;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const u64 lo = L[j], hi = L[j + H];
        a0 += -(i128)hi - (i128)lo;
        a1 += (i128)lo - (i128)hi;
        L[j] = (u64)a0;
        L[j + H] = (u64)a1;
        a0 >>= 64;
        a1 >>= 64;
    }
    i128 c = a0;
#pragma unroll
    for (int j = H; j < M; ++j) {
        c += (i128)L[j];
        L[j] = (u64)c;
        c >>= 64;
    }
    T = (int)(i64)(a1 + c);
}

// The product's limbs go to `Z`: registers (u64 (&)[M]) or, on the device, this thread's word
// column of the LDS exchange rows (PwLdsZ: limb j as words 2j, 2j + 1) -- the latter keeps the M limbs out of the
// registers while the 2 ND digits are live (the l = 4096 kernel spilled 32 VGPRs at the
// 128-VGPR budget with the limbs in registers, the l = 2048 one 5).
struct PwLdsRef {
    u32 *p;    // word 0 of the limb (its high word K further): the publish layout (pw_publish_words)
    int K;
    __device__ __forceinline__ operator u64() const { return ((u64)p[K] << 32) | p[0]; }
    __device__ __forceinline__ PwLdsRef &operator=(u64 v)
    {
        p[0] = (u32)v;
        p[K] = (u32)(v >> 32);
        return *this;
    }
};
struct PwLdsZ {
    u32 *z;    // Xw + t: this thread's own word column (the u64 rows would straddle two threads' columns)
    int K;
    __device__ __forceinline__ PwLdsRef operator[](int j) const { return PwLdsRef{z + 2 * j * K, K}; }
};

// z = a b mod p' for canonical a (La, ta), b (Lb, tb); result limbs + top (value = L + T 2^N')
template <int M, typename ZT>
__host__ __device__ __forceinline__ void pw_mulmod(ZT &&Z, int &T, const u64 (&La)[M], int ta, const u64 (&Lb)[M], int tb)
{
    if (ta | tb) {   // 2^N' == -1: the product is 1, -b or -a  (cf. mul_fft.c:3250)
        if (ta && tb) {
#pragma unroll
            for (int j = 0; j < M; ++j) Z[j] = j == 0;
            T = 0;
            return;
        }
        // -v = ~v + 1 - 2^N'  ->  limbs ~v, +1 at limb 0, top -1
        i128 acc = 1;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            acc += (i128)(~(ta ? Lb[j] : La[j]));
            Z[j] = (u64)acc;
            acc >>= 64;
        }
        T = -1 + (int)(i64)acc;
        return;
    }
    // Full product over 29-bit digits: a column sums at most ND < 64 products < 2^58,
    // so one v_mad_u64_u32 per digit product with no carry tracking.  Columns are
    // streamed into 64-bit limbs and folded on the fly: Z = lo - hi (2^N' == -1).
    constexpr int DB = 29, ND = (64 * M + DB - 1) / DB;
    static_assert(ND < 64, "column sums must stay below 2^64");
    u32 ad[ND], bd[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const int b0 = d * DB, li = b0 >> 6, sh = b0 & 63;
        u64 x = La[li] >> sh, y = Lb[li] >> sh;
        if (sh + DB > 64 && li + 1 < M) {
            x |= La[li + 1] << (64 - sh);
            y |= Lb[li + 1] << (64 - sh);
        }
        ad[d] = (u32)(x & ((1u << DB) - 1));
        bd[d] = (u32)(y & ((1u << DB) - 1));
    }
    u128 acc = 0;          // bits [pos, ...) of the product not yet emitted
    int pos = 0, k = 0;    // compile-time after unrolling
    i64 bw = 0;            // borrow of the lo - hi fold
#pragma clang loop unroll(full)
    for (int c = 0; c < 2 * ND - 1; ++c) {
        u64 col = 0;
        const int i0 = c < ND ? 0 : c - ND + 1, i1 = c < ND ? c : ND - 1;
#pragma clang loop unroll(full)
        for (int i = i0; i <= i1; ++i) col += (u64)ad[i] * bd[c - i];
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_sched_barrier(0);   // one column's products live at a time (VGPRs)
#endif
        acc += (u128)col << (DB * c - pos);
        const bool last = c == 2 * ND - 2;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            if (k < 2 * M && (last || DB * (c + 1) - pos >= 64)) {
                const u64 limb = (u64)acc;
                acc >>= 64;
                pos += 64;
                if (k < M) {
                    Z[k] = limb;
                } else {                       // fold: Z[k - M] -= limb (borrow chain)
                    const u64 z = Z[k - M];
                    const u64 d1 = z - limb;
                    i64 b1 = (i64)(d1 > z);
                    const u64 d2 = d1 + (u64)bw;   // bw <= 0
                    b1 += bw < 0 ? (i64)(d2 > d1) : 0;
                    Z[k - M] = d2;
                    bw = -b1;
                }
                ++k;
            }
        }
    }
    T = (int)bw;   // value = Z + T 2^N', T in {-1, 0}
}

// exchange: thread t publishes its value as words (normalised first: pw_norm) and, unless
// TT is null (tight form), its top
template <int M, int LK>
__device__ __forceinline__ void pw_publish_words(const u64 (&L)[M], u32 *Xw, int t)
{
    constexpr int K = 1 << LK;
    // (an opaque copy of this address, to keep the second base register of the rows past the
    // 64 KiB ds offset reach from living across the levels, cut the l = 4096 spills 84 -> 68 B
    // per lane and slowed the kernel 40.0 -> 44.5 ms: profiles/r05/pw_lds_product_ab.txt)
    u32 *col = Xw + t;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        col[(2 * j) * K] = (u32)L[j];
        col[(2 * j + 1) * K] = (u32)(L[j] >> 32);
    }
}

template <int M, int LK>
__device__ __forceinline__ void pw_publish(u64 (&L)[M], int &T, int S, u32 *Xw, int *TT, int t)
{
    T = pw_norm<M>(L, T);
    pw_publish_words<M, LK>(L, Xw, t);
    if (TT) TT[t] = 2 * T + S;
}

// One forward (DIF) or inverse (DIT) length-K cyclic transform with root 2^W2 over
// the values of the K threads of this workgroup.  P: this thread's pending exponent.
// a mod n for a < 4n, without a division (every exponent here is a sum of a few reduced terms)
__device__ __forceinline__ unsigned pw_mod(unsigned a, unsigned n)
{
    a = a >= 2 * n ? a - 2 * n : a;
    return a >= n ? a - n : a;
}

// an opaque copy of the thread index: values derived from it are recomputed where used
// instead of kept live across the transforms (cf. rp_launder)
__device__ __forceinline__ int pw_launder(int t)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(t));
#endif
    return t;
}

// Exchange ordering inside one wave: a wave's LDS instructions execute in issue order, so a
// level whose butterfly partners share a wave (h < 64) needs no workgroup barrier -- only a
// compiler fence that keeps this level's reads after its publish and before the next
// publish.  Levels with h >= 64 exchange across waves and keep both __syncthreads.
__device__ __forceinline__ void pw_wave_sync()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// the combine of a forward level j whose rotation E mod N' is one of the odd multiples of
// N' / 2^(j+1) and the same for the whole wave: a scalar switch to the compile-time rotation
// (pw_combine FIXE); anything else (never, by pw_transform's derivation) takes the general form
// (Eu = the wave's E mod N', an odd multiple (2I + 1) N' / 2^(J+1): I selects the copy; the last
// copy also takes any other value, which pw_transform's derivation rules out -- checked exactly
// for both kernel shapes by tests/test_pw_host.py's simulation of the pending exponents)
template <int M, int LK, int J, int I = 0>
__device__ __forceinline__ void pw_combine_fixed(u64 (&L)[M], int &T, int &S, int alpha, const u32 *Xw, int packed, int q,
                                                 unsigned E, unsigned Eu)
{
    constexpr unsigned NP = 64 * M;
    constexpr unsigned C = (2 * I + 1) * (NP >> (J + 1));
    if constexpr (I + 1 < (1 << J)) {
        if (Eu == C) {
            pw_combine<M, LK, pw_pd<M, LK>(), (int)C>(L, T, S, alpha, Xw, packed, q, E);
            return;
        }
        pw_combine_fixed<M, LK, J, I + 1>(L, T, S, alpha, Xw, packed, q, E, Eu);
    } else {
        pw_combine<M, LK, pw_pd<M, LK>(), (int)C>(L, T, S, alpha, Xw, packed, q, E);
    }
}

#ifndef PW_UNW_FUSE
#define PW_UNW_FUSE 1   // 0 (A/B builds): the un-weighting as its own publish + rotated read after the inverse
#endif
#ifndef PW_PROBE_NOH1
#define PW_PROBE_NOH1 0   // 1: timing probe, the h = 1 levels without their LDS round (A/B builds only)
#endif
// one level jj of the transform.  FIXJ >= 0 (forward transforms, level jj = FIXJ): E mod N' is
// wave-uniform and one of 2^FIXJ compile-time values (level 0: exactly N'/2) -- pw_transform
// UNW (the inverse's last level, h = K/2): the un-weighting theta^-t 2^-lk folded in -- with F the
// exponent it applies after the level (pw_unweight_exp), r = alpha 2^F own + 2^(E + F) x_q: own is
// read back rotated from the words it has just published for its partner, so the separate publish +
// rotated read of the un-weighting is gone (pw_slot_product)
template <int M, int LK>
__device__ __forceinline__ unsigned pw_unweight_exp(unsigned Pz, unsigned W2, int t)
{
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    // theta^-t 2^-lk: 2^-(t W2 / 2 + lk), for a half-integer t W2 / 2 (sqrt 2)^-1 = sqrt 2 / 2:
    // 2^(-floor(t W2 / 2) - 1 - lk + N'/4) (2^(N'/2) - 1) -- the (2^(N'/2) - 1) factor by the caller
    const bool halff = (W2 & 1) && (t & 1);
    const unsigned un = (((unsigned)t * W2) >> 1) + LK + (halff ? 1 : 0);   // < N' + lk + 1
    return pw_mod(Pz + N2 - un + (halff ? NP / 4 : 0), N2);
}

template <int M, int LK, int DIR, int FIXJ, bool UNW = false>
__device__ __forceinline__ void pw_level(u64 (&L)[M], int &T, int &S, unsigned &P, u32 *Xw, int *TT, unsigned *PP,
                                         unsigned W2, int t, int jj, bool unw = false)
{
    constexpr int K = 1 << LK, lk = LK;
    constexpr unsigned N2 = 128 * M;
    const int j = DIR == 0 ? jj : lk - 1 - jj;   // DIF level index (DIT runs them backwards)
    const int h = K >> (j + 1);
    const int q = t ^ h;
    const bool top = !(t & h);
    const int qt = t & ~h;                       // top index of the pair
    // (qt mod h) 2^j < K/2, times W2: below N' (= K W2 / 2): no reduction needed
    const unsigned tw = (unsigned)((qt & (h - 1)) << j) * W2;
    const bool cross = h >= 64;                  // partner in another wave
#if PW_PROBE_NOH1
    if (h == 1) {   // timing probe (A/B builds only, wrong products): the h = 1 level without its LDS round
        u64 cy = P;
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const u64 s = L[m] + cy;
            cy = s < L[m] ? 1 : 0;
            L[m] = s;
        }
        if (!top) P = pw_mod(P + 1, N2);
        return;
    }
#endif
    unsigned Pq;
    int packed;
    if (pw_tight(K)) {
        // the partner's top / sign and exponent first (a shuffle, or through rows 0-1 before
        // the words overwrite them), then the words
        T = pw_norm<M>(L, T);
        const int own = 2 * T + S;
        if (cross) {
            Xw[t] = (u32)own;
            Xw[K + t] = P;
            __syncthreads();
            packed = (int)Xw[q];
            Pq = Xw[K + q];
            __syncthreads();
        } else {
            packed = __shfl_xor(own, h);
            Pq = (unsigned)__shfl_xor((int)P, h);
        }
        pw_publish_words<M, LK>(L, Xw, t);
        if (cross) __syncthreads(); else pw_wave_sync();
    } else {
        pw_publish<M, LK>(L, T, S, Xw, TT, t);
        PP[t] = P;
        if (cross) __syncthreads(); else pw_wave_sync();
        Pq = PP[q];
        packed = TT[q];
    }
    const int own_packed = 2 * T + S;   // (UNW) as published: T normalised by pw_publish / pw_norm
    unsigned E;
    if (DIR == 0) {
        // top: X_t + X_q = 2^P (x_t + 2^(Pq-P) x_q); bottom: (X_q - X_t) w^tw = 2^(P+tw) (2^(Pq-P) x_q - x_t)
        E = pw_mod(Pq + N2 - P, N2);
        if constexpr (FIXJ == 0) {
            pw_combine<M, LK, pw_pd<M, LK>(), 32 * M>(L, T, S, top ? 1 : -1, Xw, packed, q, E);
        } else if constexpr (FIXJ > 0) {
            constexpr unsigned NP = 64 * M;
            const unsigned Em = E >= NP ? E - NP : E;
            const unsigned Eu = (unsigned)__builtin_amdgcn_readfirstlane((int)Em);   // wave-uniform (above)
            pw_combine_fixed<M, LK, FIXJ>(L, T, S, top ? 1 : -1, Xw, packed, q, E, Eu);
        } else {
            pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, top ? 1 : -1, Xw, packed, q, E);
        }
        if (!top) P = pw_mod(P + tw, N2);
    } else {
        // top: Z_t + Z_q w^-tw = 2^P (z_t + 2^(Pq-tw-P) z_q)
        // bottom: Z_q - Z_t w^-tw = 2^(P-tw) (2^(Pq-P+tw) z_q - z_t)
        E = top ? pw_mod(Pq + 2 * N2 - tw - P, N2) : pw_mod(Pq + N2 - P + tw, N2);
        if (UNW && unw) {
            if (!top) P = pw_mod(P + N2 - tw, N2);
            const unsigned F = pw_unweight_exp<M, LK>(P, W2, pw_tight(K) ? pw_launder(t) : t);
            constexpr unsigned NP = 64 * M;
            const unsigned Eq = pw_mod(E + F, N2);
            pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, 0, Xw, own_packed, t, top ? F : pw_mod(F + NP, N2));
            __builtin_amdgcn_sched_barrier(0);   // the two rotated reads one after the other
            pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, 1, Xw, packed, q, Eq);
            P = 0;
        } else {
            pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, top ? 1 : -1, Xw, packed, q, E);
            if (!top) P = pw_mod(P + N2 - tw, N2);
        }
    }
    if (cross) __syncthreads(); else pw_wave_sync();
}

// Two DIT levels per exchange (A/B builds: -DPW_R4_INV=1): levels jj (pairs h1 =
// K >> (lk - jj)) and jj + 1 (h2 = 2 h1) on the quad t0 | {0, h1, h2, h1 + h2} of role i = [t & h1]
// + 2 [t & h2], from one publish: with A, B_i the two levels' twiddles (B_i that of the level-(jj+1)
// pair holding t) every output is v_i = sum_r sigma_ir w^-e_ir Z_r, e_i0 = 0, e_i1 = A, e_i2 = B_i,
// e_i3 = A + B_i, sigma_i1 = -[i odd], sigma_i2 = -[i >= 2], sigma_i3 = sigma_i1 sigma_i2 -- own term
// plus three rotated partner reads (pw_combine), one barrier pair instead of two.  Same LDS traffic
// (one 2M-word publish + three reads against two + two), 1.5x the add chains.
#ifndef PW_R4_INV
#define PW_R4_INV 0
#endif
template <int M, int LK>
__device__ __forceinline__ void pw_level4_dit(u64 (&L)[M], int &T, int &S, unsigned &P, u32 *Xw, int *TT, unsigned *PP,
                                              unsigned W2, int t, int jj)
{
    constexpr int K = 1 << LK;
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    static_assert(!pw_tight(K), "the radix-4 levels use the TT / PP arrays");
    const int jA = LK - 1 - jj, jB = jA - 1;
    const int h1 = K >> (jA + 1), h2 = 2 * h1;
    const int role = ((t & h1) ? 1 : 0) | ((t & h2) ? 2 : 0);
    const int t0 = t & ~(h1 | h2);
    const unsigned A = (unsigned)((t & (h1 - 1)) << jA) * W2;   // < N' (as pw_level's tw)
    const unsigned B = (unsigned)((t & (h2 - 1)) << jB) * W2;
    const bool cross = h2 >= 64;
    pw_publish<M, LK>(L, T, S, Xw, TT, t);
    PP[t] = P;
    if (cross) __syncthreads(); else pw_wave_sync();
    const unsigned eA = A ? N2 - A : 0u, eB = B ? N2 - B : 0u;
    auto ex = [&](int r) -> unsigned { return r == 0 ? 0u : r == 1 ? eA : r == 2 ? eB : pw_mod(eA + eB, N2); };
    const bool n1 = role & 1, n2 = (role >> 1) & 1;
    auto neg = [&](int r) -> bool { return r == 0 ? false : r == 1 ? n1 : r == 2 ? n2 : n1 != n2; };
    const unsigned Pn = pw_mod(P + ex(role), N2);
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const int r = role ^ k;
        const int q = t0 | ((r & 1) ? h1 : 0) | ((r & 2) ? h2 : 0);
        const unsigned Pq = PP[q];
        const int packed = TT[q];
        unsigned E = pw_mod(Pq + ex(r) + 2 * N2 - Pn, N2);
        if (neg(r)) E = pw_mod(E + NP, N2);
        pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, k == 1 ? (neg(role) ? -1 : 1) : 1, Xw, packed, q, E);
    }
    P = Pn;
    if (cross) __syncthreads(); else pw_wave_sync();
}

// The same for two DIF levels (A/B builds: -DPW_R4_FWD=1): levels jj (h1 = K >> (jj + 1)) and
// jj + 1 (h2 = h1 / 2), role i = [t & h2] + 2 [t & h1]; with a_r = ((t0 | [r odd] h2) mod h1) 2^jj W2
// and B = (t0 mod h2) 2^(jj+1) W2, v_i = sum_r (-1)^popcount(i & r) w^e_ir X_r,
// e_ir = [i odd] B + [i >= 2] a_r.
#ifndef PW_R4_FWD
#define PW_R4_FWD 0
#endif
template <int M, int LK>
__device__ __forceinline__ void pw_level4_dif(u64 (&L)[M], int &T, int &S, unsigned &P, u32 *Xw, int *TT, unsigned *PP,
                                              unsigned W2, int t, int jj)
{
    constexpr int K = 1 << LK;
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    static_assert(!pw_tight(K), "the radix-4 levels use the TT / PP arrays");
    const int h1 = K >> (jj + 1), h2 = h1 / 2;
    const int role = ((t & h2) ? 1 : 0) | ((t & h1) ? 2 : 0);
    const int t0 = t & ~(h1 | h2);
    const unsigned a0 = (unsigned)((t0 & (h1 - 1)) << jj) * W2, a1 = (unsigned)(((t0 | h2) & (h1 - 1)) << jj) * W2;
    const unsigned B = (unsigned)((t0 & (h2 - 1)) << (jj + 1)) * W2;
    const bool cross = h1 >= 64;
    pw_publish<M, LK>(L, T, S, Xw, TT, t);
    PP[t] = P;
    if (cross) __syncthreads(); else pw_wave_sync();
    auto ex = [&](int i, int r) -> unsigned {
        return pw_mod(((i & 1) ? B : 0u) + ((i & 2) ? ((r & 1) ? a1 : a0) : 0u), N2);
    };
    auto neg = [&](int i, int r) -> bool { return __builtin_popcount(i & r) & 1; };
    const unsigned Pn = pw_mod(P + ex(role, role), N2);
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const int r = role ^ k;
        const int q = t0 | ((r & 1) ? h2 : 0) | ((r & 2) ? h1 : 0);
        const unsigned Pq = PP[q];
        const int packed = TT[q];
        unsigned E = pw_mod(Pq + ex(role, r) + 2 * N2 - Pn, N2);
        if (neg(role, r)) E = pw_mod(E + NP, N2);
        pw_combine<M, LK, pw_pd<M, LK>()>(L, T, S, k == 1 ? (neg(role, role) ? -1 : 1) : 1, Xw, packed, q, E);
    }
    P = Pn;
    if (cross) __syncthreads(); else pw_wave_sync();
}

// the highest compile-time-rotation level of operand B's transform in the late-B (l = 4096) form:
// level 0 only -- while B transforms, A's transformed limbs are live, and the switch copies of
// levels 1 and 2 pushed the kernel into spilling (96 -> 40 B per lane; C4 pointwise 34.0 -> 32.3 ms,
// levels 0-1: 32.6; profiles/r05/pw_fixb_ab.txt).  A/B builds: -DPW_FIXB=1 / 2
#ifndef PW_FIXB
#define PW_FIXB 0
#endif
#ifndef PW_FIXB_EARLY
#define PW_FIXB_EARLY 2   // A/B builds: the same for operand B loaded with A (l <= 2048)
#endif
template <int M, int LK, int DIR, int FIXMAX = 2>
__device__ __forceinline__ void pw_transform(u64 (&L)[M], int &T, int &S, unsigned &P, u32 *Xw, int *TT, unsigned *PP,
                                             unsigned W2, int t)
{
    int jj = 0;
    if (DIR == 0) {
        // The forward levels' rotations at the top of the DIF.  Before level j, P_t is the weight
        // floor(t W2 / 2) (+ N'/4 for a half exponent: equal for t and its partner q = t ^ h_j) plus,
        // for every earlier level j' whose bit h_j' = K >> (j'+1) t has, the twiddle
        // ((t mod h_j') << j') W2.  q differs from t in bit h_j only, so
        //   E = Pq - P = +-[h_j W2 / 2 + sum_(j' < j, bit h_j' of t) (h_j << j') W2]
        //     = +-[N' / 2^(j+1) + sum N' / 2^(j - j')]   (K W2 = 2 N'),
        // an odd multiple of N' / 2^(j+1), fixed by the bits h_0 .. h_(j-1) of t and the sign by
        // bit h_j: wave-uniform while h_j >= 64.  Level 0: exactly N'/2 for every thread; levels
        // 1 .. log2(K/128): one of 2^j values, a scalar switch to the compile-time rotation (the
        // per-word wrap tests, addresses and complement masks fold away).  Each level is its own
        // inlined copy (peeled off the loop: one loop body with both forms spilled 3x more).
        static_assert(LK >= 7, "level 0's partner K/2 >= 64 lanes away");
        pw_level<M, LK, DIR, 0>(L, T, S, P, Xw, TT, PP, W2, t, 0);
        if constexpr (LK >= 8 && FIXMAX >= 1) pw_level<M, LK, DIR, 1>(L, T, S, P, Xw, TT, PP, W2, t, 1);   // h = K/4 >= 64
        if constexpr (LK >= 9 && FIXMAX >= 2) pw_level<M, LK, DIR, 2>(L, T, S, P, Xw, TT, PP, W2, t, 2);   // h = K/8 >= 64
        jj = LK >= 9 && FIXMAX >= 2 ? 3 : LK >= 8 && FIXMAX >= 1 ? 2 : 1;
    }
    if constexpr (DIR == 1 && PW_R4_INV && !pw_tight(1 << LK)) {
        for (; jj + 1 < LK; jj += 2) pw_level4_dit<M, LK>(L, T, S, P, Xw, TT, PP, W2, t, jj);
    }
    if constexpr (DIR == 0 && PW_R4_FWD && !pw_tight(1 << LK)) {
        for (; jj + 1 < LK; jj += 2) pw_level4_dif<M, LK>(L, T, S, P, Xw, TT, PP, W2, t, jj);
    }
    for (; jj < LK; ++jj) pw_level<M, LK, DIR, -1, DIR == 1 && PW_UNW_FUSE>(L, T, S, P, Xw, TT, PP, W2, t, jj, jj == LK - 1);
}

// Piece t of a coefficient in the reduced HBM form (coeff.hpp: limbs + carry masks +
// carry limb): limbs [t LP, t LP + LP) plus the carries into them -- the carry out of
// limb m lands in limb m + 1, the carry into limb 0 is minus the carry out of limb l-1
// and minus the carry limb (both weigh 2^N == -1); the carry out of the piece's top limb
// is the next piece's.  The value v (-2 <= v < 2^(64 LP) + 2^(64 LP - 64)) is returned as
// L + T 2^N', T in {-1, 0}: the convolution tolerates such pieces (|c_t| < K 2^(2B+1)
// still fits the headroom N' >= 2B + lk + 4, pdispatch.hpp), so the pointwise inputs need no
// canonicalisation pass.  A piece lies inside one 64-limb mask row (LP | 64).
// The loads of a piece (its LP limbs, its own carry-mask words and those of the limb below
// it, the slot's carry limb), issued before any of them is used (pw_piece_fetch), then the
// arithmetic (pw_piece_make): a workgroup requests all its pieces' bytes at once and waits
// one HBM round trip, where a load-compute-load order waited one per piece (the masks of
// the limb below depend on nothing loaded, so nothing forces the order).
template <int LP>
struct PwRaw {
    u64 v[LP];
    u64 pw, nw;     // carry masks of the piece's 64-limb row
    u64 pwp, nwp;   // of the row holding limb m0 - 1 (or l - 1 for piece 0)
    int top;
};

template <int LP>
__device__ __forceinline__ void pw_piece_fetch(PwRaw<LP> &R, const u64 *dig, const u64 *cbp, const int *topp, int l,
                                               int t)
{
    typedef unsigned long long pw_v2u __attribute__((ext_vector_type(2)));
    static_assert(LP % 2 == 0, "pieces of whole limb pairs");
    const int m0 = t * LP, W = m0 >> 6, mb = m0 ? m0 - 1 : l - 1, Wp = mb >> 6;
    // the piece's LP limbs as 16-byte loads (m0 even, slots 64-byte aligned)
#pragma unroll
    for (int j = 0; j < LP; j += 2) {
        const pw_v2u q = *(const pw_v2u *)(dig + m0 + j);
        R.v[j] = q.x;
        R.v[j + 1] = q.y;
    }
    const pw_v2u c = *(const pw_v2u *)(cbp + 2 * W), cp = *(const pw_v2u *)(cbp + 2 * Wp);
    R.pw = c.x;
    R.nw = c.y;
    R.pwp = cp.x;
    R.nwp = cp.y;
    R.top = *topp;
}

// Piece t of a coefficient in the reduced HBM form (coeff.hpp: limbs + carry masks +
// carry limb): limbs [t LP, t LP + LP) plus the carries into them -- the carry out of
// limb m lands in limb m + 1, the carry into limb 0 is minus the carry out of limb l-1
// and minus the carry limb (both weigh 2^N == -1); the carry out of the piece's top limb
// is the next piece's.  The value v (-2 <= v < 2^(64 LP) + 2^(64 LP - 64)) is returned as
// L + T 2^N', T in {-1, 0}: the convolution tolerates such pieces (|c_t| < K 2^(2B+1)
// still fits the headroom N' >= 2B + lk + 4, pdispatch.hpp), so the pointwise inputs need no
// canonicalisation pass.  A piece lies inside one 64-limb mask row (LP | 64).
template <int M, int LP>
__device__ __forceinline__ void pw_piece_make(u64 (&L)[M], int &T, const PwRaw<LP> &R, int l, int t)
{
    const int m0 = t * LP, b0 = m0 & 63;
    const int mb = m0 ? m0 - 1 : l - 1, bp = mb & 63;
    const int kb = (int)((R.pwp >> bp) & 1) - (int)((R.nwp >> bp) & 1);
    const int cin = m0 ? kb : -kb - R.top;
    i64 c = cin;   // signed carry into the next limb
#pragma unroll
    for (int j = 0; j < LP; ++j) {
        const u64 v = R.v[j];
        const int k = j ? (int)((R.pw >> (b0 + j - 1)) & 1) - (int)((R.nw >> (b0 + j - 1)) & 1) : 0;
        const i64 add = c + k;        // |add| <= 4
        const u64 r = v + (u64)add;
        c = add >= 0 ? (i64)(r < v) : -(i64)(r > v);
        L[j] = r;
    }
    // the carry c out of limb LP - 1 in {-1, 0, 1}: limb LP = c, sign-extended above (one
    // register for all the upper limbs), top -1 for a negative piece
    const u64 up = c < 0 ? ~0ull : 0ull;
#pragma unroll
    for (int j = LP; j < M; ++j) L[j] = j == LP ? (c > 0 ? 1ull : up) : up;
    T = c < 0 ? -1 : 0;
}

template <int M, int LP>
__device__ __forceinline__ void pw_load_piece(u64 (&L)[M], int &T, const u64 *dig, const u64 *cbp, const int *topp,
                                              int l, int t)
{
    PwRaw<LP> R;
    pw_piece_fetch<LP>(R, dig, cbp, topp, l, t);
    pw_piece_make<M, LP>(L, T, R, l, t);
}

// limbs per piece of the instantiated k_pwss shapes: l / K (l = 1024: M = 10, LP = 4;
// l = 2048, 4096: M = 18, 20, LP = 8)
template <int M, int LK>
__host__ __device__ constexpr int pw_piece_limbs() { return M <= 12 ? 4 : 8; }

// Piece t of x0 + x1 (sub = 0) or x0 - x1 (sub = 1) for two reduced-form coefficients: the
// last DIF level of the row transform (h = 1, twiddle 1) applied piecewise -- linear, so the
// pieces of the sum / difference are the sums / differences of the pieces (|c_t| at most
// doubles: the headroom N' >= 2B + lk + 4 covers it, pdispatch.hpp).  Each piece is LP limbs plus a carry
// in {-1, 0, 1} (pw_load_piece); the LP + 1 limb result is sign-extended to M limbs, T = -1
// for a negative value.
template <int M, int LP>
__device__ __forceinline__ void pw_load_pair_bfly(u64 (&L)[M], int &T, const u64 *dig, const u64 *cb, const int *top,
                                                  long s0, int l, int cbw, int t, bool sub)
{
    u64 A[M], B[M];
    int Ta, Tb;
    {
        PwRaw<LP> RA, RB;   // both slots' bytes requested before either is used
        pw_piece_fetch<LP>(RA, dig + (size_t)s0 * l, cb + (size_t)s0 * cbw, top + s0, l, t);
        pw_piece_fetch<LP>(RB, dig + (size_t)(s0 + 1) * l, cb + (size_t)(s0 + 1) * cbw, top + s0 + 1, l, t);
        pw_piece_make<M, LP>(A, Ta, RA, l, t);
        pw_piece_make<M, LP>(B, Tb, RB, l, t);
    }
    // limbs LP .. M-1 of A, B are the sign extension (carry limb LP, then 0 / ~0): add LP + 1 limbs
    const u32 m = sub ? ~0u : 0u;
    u32 c = sub ? 1u : 0u;
#pragma unroll
    for (int j = 0; j <= LP; ++j) {
        const u32 lo = __builtin_addc((u32)A[j], (u32)B[j] ^ m, c, &c);
        const u32 hi = __builtin_addc((u32)(A[j] >> 32), (u32)(B[j] >> 32) ^ m, c, &c);
        L[j] = ((u64)hi << 32) | lo;
    }
    // the values are below 2^(64 LP + 2) in magnitude: limb LP's sign is the result's sign
    const u64 up = (i64)L[LP] < 0 ? ~0ull : 0ull;
#pragma unroll
    for (int j = LP + 1; j < M; ++j) L[j] = up;
    T = (i64)L[LP] < 0 ? -1 : 0;
    (void)Ta;
    (void)Tb;
}

// Piece t of output pos (0..3) of the row DIF's last two levels on the slot quad x0..x3
// (positions 4i..4i+3 of a row, the levels h = 2 and h = 1 of a length-NC DIF with root
// 2^(w NR)): z0 = (x0 + x2) + (x1 + x3), z1 = (x0 + x2) - (x1 + x3), z2 = (x0 - x2) + w (x1 - x3),
// z3 = (x0 - x2) - w (x1 - x3), with w = 2^(w NR NC / 4) = 2^(N/2): piece t of 2^(N/2) v is
// piece t ^ K/2 of v, negated for t < K/2 (2^N == -1) -- a load address, not arithmetic.
// Linear, so the pieces of z are signed sums of the inputs' pieces (|c_t| grows 4x: the inner
// ring's headroom covers it, pdispatch.hpp).  Sums are kept in LP + 1 limbs two's complement,
// one input piece formed at a time (registers), then sign-extended to M limbs.
template <int M, int LP, int K, int INFL = 2>
__device__ __forceinline__ void pw_load_quad_bfly(u64 (&L)[M], int &T, const u64 *dig, const u64 *cb, const int *top,
                                                  long s0, int pos, int l, int cbw, int t)
{
    u64 acc[LP + 1];
#pragma unroll
    for (int j = 0; j <= LP; ++j) acc[j] = 0;
    const int tr = t ^ (K / 2), sg = t >= K / 2 ? 1 : -1;
    // sign of input slot q in output pos; x1, x3 come from the rotated piece for pos >= 2
    auto sign_of = [&](int q) {
        return q == 0 ? 1 : q == 2 ? (pos < 2 ? 1 : -1)
             : (pos < 2 ? (pos == 0 ? 1 : -1) : (pos == 2 ? sg : -sg) * (q == 1 ? 1 : -1));
    };
    auto add = [&](const PwRaw<LP> &R, int q, int pt) {
        u64 X[M];
        int Tx;
        pw_piece_make<M, LP>(X, Tx, R, l, pt);
        // acc += sign * (limbs 0 .. LP of X): limb LP of X is the piece's carry, sign-extended
        const u32 m = sign_of(q) < 0 ? ~0u : 0u;
        u32 c = m & 1u;
#pragma unroll
        for (int j = 0; j <= LP; ++j) {
            const u32 lo = __builtin_addc((u32)acc[j], (u32)X[j] ^ m, c, &c);
            const u32 hi = __builtin_addc((u32)(acc[j] >> 32), (u32)(X[j] >> 32) ^ m, c, &c);
            acc[j] = ((u64)hi << 32) | lo;
        }
    };
    if (PW_QUAD4 || INFL == 4) {   // all four inputs' bytes in flight at once
        const int pr = pos >= 2 ? tr : t;
        PwRaw<LP> R0, R1, R2, R3;
        pw_piece_fetch<LP>(R0, dig + (size_t)s0 * l, cb + (size_t)s0 * cbw, top + s0, l, t);
        pw_piece_fetch<LP>(R2, dig + (size_t)(s0 + 2) * l, cb + (size_t)(s0 + 2) * cbw, top + s0 + 2, l, t);
        pw_piece_fetch<LP>(R1, dig + (size_t)(s0 + 1) * l, cb + (size_t)(s0 + 1) * cbw, top + s0 + 1, l, pr);
        pw_piece_fetch<LP>(R3, dig + (size_t)(s0 + 3) * l, cb + (size_t)(s0 + 3) * cbw, top + s0 + 3, l, pr);
        add(R0, 0, t);
        add(R2, 2, t);
        add(R1, 1, pr);
        add(R3, 3, pr);
    } else if (INFL == 1) {   // one input's bytes at a time (x0, x2, x1, x3)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = u < 2 ? 2 * u : 2 * (u - 2) + 1, pt = (q & 1) && pos >= 2 ? tr : t;
            PwRaw<LP> R;
            pw_piece_fetch<LP>(R, dig + (size_t)(s0 + q) * l, cb + (size_t)(s0 + q) * cbw, top + s0 + q, l, pt);
            add(R, q, pt);
        }
    } else
    // two inputs' bytes in flight at a time (x0, x2 at piece t; then x1, x3)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int qa = h, qb = h + 2, pt = h && pos >= 2 ? tr : t;
        PwRaw<LP> Ra, Rb;
        pw_piece_fetch<LP>(Ra, dig + (size_t)(s0 + qa) * l, cb + (size_t)(s0 + qa) * cbw, top + s0 + qa, l, pt);
        pw_piece_fetch<LP>(Rb, dig + (size_t)(s0 + qb) * l, cb + (size_t)(s0 + qb) * cbw, top + s0 + qb, l, pt);
        add(Ra, qa, pt);
        add(Rb, qb, pt);
    }
    // |sum| < 2^(64 LP + 3): limb LP's sign is the value's sign
    const u64 up = (i64)acc[LP] < 0 ? ~0ull : 0ull;
#pragma unroll
    for (int j = 0; j < M; ++j) L[j] = j <= LP ? acc[j] : up;
    T = (i64)acc[LP] < 0 ? -1 : 0;
}

// inner product of one slot: forward transforms of the pieces (La, Ta), (Lb, Tb), the
// pointwise products in R', the inverse and the un-weighting; leaves the signed
// coefficients c_t in X (limb-major, M rows) and their signs (+ limb M) in TT (ends with a barrier)
// loadB(Lb, Tb): when given (the tight form), operand B's pieces are loaded only after A's
// forward transform, so the two operands' raw and formed pieces are never live together (the
// kernel's register peak at 128 VGPRs; B's load latency is hidden by the CU's other workgroup)
template <int M, int LK, typename LoadB = int>
__device__ __forceinline__ void pw_slot_product(u64 (&La)[M], int Ta, u64 (&Lb)[M], int Tb, u64 *X, u32 *Xw, int *TT,
                                                unsigned *PP, int t, unsigned long long *stamp, LoadB loadB = 0)
{
    constexpr bool late_b = !std::is_same<LoadB, int>::value;
#define PW_STAMP(k) do { if (stamp && t == 0) stamp[k] = __builtin_amdgcn_s_memtime(); } while (0)
    constexpr int K = 1 << LK, lk = LK;
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    constexpr unsigned W2 = N2 >> lk;            // omega = 2^W2 (host: K / 2 divides N')
    static_assert((N2 >> lk) << lk == N2, "omega must be a power of two");
    int Sa = 0, Sb = 0;                          // sign flags
    // negacyclic weight theta^t = 2^(t W2 / 2); a half-integer exponent (W2 and t odd) is
    // 2^(floor(t W2 / 2) + N'/4) (2^(N'/2) - 1)  (sqrt 2 = 2^(N'/4) (2^(N'/2) - 1) in R').
    // Recomputed from an opaque copy of t where used again at l = 4096 (pw_launder): kept live
    // from here to the un-weighting they took VGPRs that kernel spilled (144 -> 96 B per lane,
    // C4 pointwise 35.8 -> 34.9 ms)
    auto weight = [&](int tt) -> unsigned {
        return (((unsigned)tt * W2) >> 1) + (((W2 & 1) && (tt & 1)) ? NP / 4 : 0);   // < N' + N'/4
    };
    const bool half = (W2 & 1) && (t & 1);
    unsigned Pa = weight(t), Pb = late_b ? 0u : Pa;
    if (half) {
        pw_sqrt2<M>(La, Ta);
        if (!late_b) pw_sqrt2<M>(Lb, Tb);
    }
    PW_STAMP(1);
    pw_transform<M, LK, 0>(La, Ta, Sa, Pa, Xw, TT, PP, W2, t);
    PW_STAMP(2);
    if constexpr (late_b) {
        loadB(Lb, Tb);
        const int tb = pw_launder(t);
        Pb = weight(tb);
        if ((W2 & 1) && (tb & 1)) pw_sqrt2<M>(Lb, Tb);
    }
    pw_transform<M, LK, 0, late_b ? PW_FIXB : PW_FIXB_EARLY>(Lb, Tb, Sb, Pb, Xw, TT, PP, W2, t);
    PW_STAMP(3);

    // ---- inner products: 2^Pa xa * 2^Pb xb = 2^(Pa + Pb) (xa xb) ---------------------
    const int ca = pw_canon<M>(La, Ta), cb = pw_canon<M>(Lb, Tb);
    u64 Z[M];
    int Tz, Sz = Sa ^ Sb;
    if (pw_tight(K)) {
        // the product's limbs through this thread's own LDS word column (B's transform ended
        // with an in-wave level: no other wave reads this column; the inverse's first publish
        // comes after): C4 pointwise 40.5 -> 40.0 ms, its spills 128 -> 84 B per lane; at
        // l = 2048 (no spills either way) the register form is faster (3.57 vs 3.67 ms),
        // profiles/r05/pw_lds_product_ab.txt
        pw_mulmod<M>(PwLdsZ{Xw + t, K}, Tz, La, ca, Lb, cb);
#pragma unroll
        for (int j = 0; j < M; ++j) Z[j] = ((u64)Xw[(2 * j + 1) * K + t] << 32) | Xw[2 * j * K + t];
    } else {
        pw_mulmod<M>(Z, Tz, La, ca, Lb, cb);
    }
    unsigned Pz = pw_mod(Pa + Pb, N2);
    PW_STAMP(4);

    // ---- inverse, then 2^-lk (division by K) and theta^-t --------------------------
    pw_transform<M, LK, 1>(Z, Tz, Sz, Pz, Xw, TT, PP, W2, t);
    PW_STAMP(5);
    if constexpr (PW_UNW_FUSE && !(PW_R4_INV && !pw_tight(K) && LK % 2 == 0)) {
        // the rotation by theta^-t 2^-lk rode in the last level (pw_level UNW); the (2^(N'/2) - 1)
        // of a half-integer weight commutes with it (that level ended with a barrier: the u64 rows
        // below may cross columns)
        const int tf = pw_tight(K) ? pw_launder(t) : t;
        if ((W2 & 1) && (tf & 1)) pw_sqrt2<M>(Z, Tz);
    } else {
        // theta^-t 2^-lk: 2^-(t W2 / 2 + lk), for a half-integer t W2 / 2 (sqrt 2)^-1 = sqrt 2 / 2:
        // 2^(-floor(t W2 / 2) - 1 - lk + N'/4) (2^(N'/2) - 1)
        const int tf = pw_tight(K) ? pw_launder(t) : t;   // (at l = 2048 the laundered form measured 1 % slower)
        const bool halff = (W2 & 1) && (tf & 1);
        const unsigned un = (((unsigned)tf * W2) >> 1) + lk + (halff ? 1 : 0);   // < N' + lk + 1
        const unsigned F = pw_mod(Pz + N2 - un + (halff ? NP / 4 : 0), N2);
        if (halff) pw_sqrt2<M>(Z, Tz);
        pw_publish<M, LK>(Z, Tz, Sz, Xw, pw_tight(K) ? nullptr : TT, t);
        pw_wave_sync();                                  // own column only
        pw_combine<M, LK, pw_pd<M, LK>()>(Z, Tz, Sz, 0, Xw, 2 * Tz + Sz, t, F);   // clears the sign flag
        __syncthreads();                                 // the u64 rows below cross columns
    }
    // signed coefficient c_t = v - s p', v in [0, 2^N'], s = (v > 2^(N'-1))
    const int zt = pw_canon<M>(Z, Tz);
    const int neg = zt || (Z[M - 1] >> 63);
    if (pw_tight(K)) {
        // as N'-bit two's complement: v - s (v - 1 = 2^N' - 1 for v = 2^N'), its top bit the sign
        u64 b = (u64)neg;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const u64 z = Z[j];
            X[j * K + t] = z - b;
            b = b && z == 0;
        }
    } else {
#pragma unroll
        for (int j = 0; j < M; ++j) X[j * K + t] = Z[j];
        TT[t] = neg | (zt << 1);                     // s, and limb M of v (2^N' only)
    }
    __syncthreads();
    PW_STAMP(6);
#undef PW_STAMP
}

// R = sum_t c_t 2^(B t) mod 2^N + 1 from X / TT, stored in the reduced HBM form at
// (pa, cbp, *topp).  c_t 2^(Bt) = v_t 2^(Bt) - s_t (2^(Bt) + 2^(N' + Bt)); positions >= N
// wrap negated.  Thread t of NTH sums output limbs m = t + NTH r (coalesced, consecutive
// per wave).  H (the l limb overflows) aliases X: written after a barrier.
template <int M, int LK, int NTH = (1 << LK)>
__device__ __forceinline__ void pw_slot_output(const u64 *X, const int *TT, int *H, u64 *pa, u64 *cbp, int *topp, int l,
                                               int t)
{
    constexpr int K = 1 << LK;
    const int LP = l >> LK;                      // limbs per piece
    const int lane = t & 63;
    u64 fo[8];
    int ho[8];
    const int RPT = l / NTH;   // <= 8 (host)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        fo[r] = 0;
        ho[r] = 0;
        if (r >= RPT) continue;
        const int m = t + NTH * r;
        i128 S = 0;
        // limb d of c_tp (0 .. M): two's complement in the tight form (limb M the sign extension)
        auto limb_of = [&](int d, int tp) -> i128 {
            i128 v;
            if (pw_tight(K)) {
                v = d < M ? (i128)X[(size_t)d * K + tp] : -(i128)(X[(size_t)(M - 1) * K + tp] >> 63);
            } else {
                const int tt = TT[tp];
                v = d < M ? (i128)X[(size_t)d * K + tp] : (i128)(tt >> 1);
                if ((tt & 1) && (d == 0 || d == M)) v -= 1;
            }
            return v;
        };
        // pieces whose limbs [t'LP, t'LP + M] cover m: t' = m / LP - j, j < M / LP + 1 -- a
        // fixed-trip loop of guarded reads (a runtime-bounded one serialised its LDS round trips)
        {
            constexpr int LPc = pw_piece_limbs<M, LK>(), KP = M / LPc + 1;
            const int hi = m / LPc;
#pragma unroll
            for (int j = 0; j < KP; ++j) {
                const int tp = hi - j, d = m - tp * LPc;
                if (tp >= 0 && d <= M) S += limb_of(d, tp);
            }
        }
        // ... and through the wrap (limb m + l, negated): only m < M
        if (m < M) {
            const int mm = m + l;
            int lo = (mm - M + LP - 1) / LP;
            for (int tp = lo; tp <= K - 1; ++tp) S -= limb_of(mm - tp * LP, tp);
        }
        fo[r] = (u64)S;
        ho[r] = (int)(i64)(S >> 64);
    }
    __syncthreads();   // every X read done: H overwrites its first rows
#pragma unroll
    for (int r = 0; r < 8; ++r)
        if (r < RPT) H[t + NTH * r] = ho[r];
    __syncthreads();
    // limb m: f_m + hv_(m-1) -> limb + carry out in {-1, 0, 1} (reduced form; the top
    // limb's overflow wraps into limb 0 negated, and its carry weighs 2^N == -1)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >= RPT) continue;
        const int m = t + NTH * r;
        const int hin = m ? H[m - 1] : -H[l - 1];
        const u64 f = fo[r];
        const u64 nf = f + (u64)(i64)hin;
        const int kout = hin >= 0 ? (int)(nf < f) : -(int)(nf > f);
        pa[m] = nf;
        const u64 pm = __ballot(kout == 1), nm = __ballot(kout == -1);
        if (lane == 0) {
            cbp[2 * (m >> 6)] = pm;
            cbp[2 * (m >> 6) + 1] = nm;
        }
    }
    if (t == 0) *topp = 0;
}

// k_pwss<M, LK, FUSE>: A[slot] <- A[slot] * B[slot] mod 2^N + 1, one workgroup of K = 2^lk
// threads per slot; reduced-form inputs and output (HBM format of coeff.hpp).
// FUSE 1: the inputs are the slot pairs (2i, 2i+1) of a row *before* the last level of the
// forward row DIF (h = 1, twiddle 1); workgroup s forms the pieces of x0 + x1 (s even) or
// x0 - x1 (s odd) of both operands on load, so that level costs no HBM pass of its own
// (mul_fft.c:2392-2408's last FFT_radix2 level fused into the pointwise loop :3244-3253,
// cf. the reference's row/pointwise fusion IFFT_radix2_mfa_truncate_sqrt2_combined :2745).
// Both workgroups of a pair read all four inputs, so the product goes to C, not in place.
// FUSE 2: the last two levels on slot quads (pw_load_quad_bfly), the four workgroups of a quad
// on one XCD.
// (Fusing the inverse row DIT's first level as well needs both products in one workgroup:
// measured at 194-256 VGPRs, occupancy 2 -> 1, so the inverse side stays a pass.)
template <int M, int LK, int FUSE>
__global__ __launch_bounds__(1 << LK) __attribute__((amdgpu_waves_per_eu(pw_wpe<M, LK>()))) void k_pwss(u64 *digA, u64 *cbA, int *topA, const u64 *digB, const u64 *cbB,
                                                  const int *topB, int l, u64 *digC, u64 *cbC, int *topC,
                                                  unsigned long long *dbg)
{
    // diagnostics (MPFFT_PW_STAMPS): thread 0 stamps the phase boundaries of this workgroup
    unsigned long long *stamp = dbg ? dbg + 8 * (size_t)blockIdx.x : nullptr;
    if (stamp && threadIdx.x == 0) stamp[0] = __builtin_amdgcn_s_memtime();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int K = 1 << LK;
    const int t = threadIdx.x;
    u64 *X = (u64 *)smem;                        // M K limbs (2M word rows during the transforms)
    u32 *Xw = (u32 *)smem;
    int *TT = pw_tight(K) ? nullptr : (int *)(X + (size_t)M * K);    // K (none in the tight form)
    unsigned *PP = pw_tight(K) ? nullptr : (unsigned *)(TT + K);     // K
    int *H = (int *)smem;                        // l, over X (pw_slot_output)
    const int cbw = cb_words(l);
    constexpr int CLP = pw_piece_limbs<M, LK>();   // == l / K (host: pw_inner_limbs)
    u64 La[M], Lb[M];
    int Ta = 0, Tb = 0;
    if (FUSE == 0 && pw_late_b(K)) {
        const long slot = blockIdx.x;
        pw_load_piece<M, CLP>(La, Ta, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA + slot, l, t);
        auto loadB = [&](u64 (&L)[M], int &T) {
            pw_load_piece<M, CLP>(L, T, digB + (size_t)slot * l, cbB + (size_t)slot * cbw, topB + slot, l, t);
        };
        pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp, loadB);
        // every piece of A was read before the first barrier of A's transform: the output may
        // overwrite A in place
        pw_slot_output<M, LK>(X, TT, H, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA + slot, l, t);
    } else if (FUSE == 0) {
        const long slot = blockIdx.x;
        {
            PwRaw<CLP> RA, RB;   // both operands' bytes requested before either is used
            pw_piece_fetch<CLP>(RA, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA + slot, l, t);
            pw_piece_fetch<CLP>(RB, digB + (size_t)slot * l, cbB + (size_t)slot * cbw, topB + slot, l, t);
            pw_piece_make<M, CLP>(La, Ta, RA, l, t);
            pw_piece_make<M, CLP>(Lb, Tb, RB, l, t);
        }
        __syncthreads();   // every piece read before any output limb is written (in place on A)
        pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp);
        pw_slot_output<M, LK>(X, TT, H, digA + (size_t)slot * l, cbA + (size_t)slot * cbw, topA + slot, l, t);
    } else if (FUSE == 2) {
        // the row DIF's last two levels on load, slot quads: blocks b, b + 8, b + 16, b + 24 take
        // the four slots of one quad, so they run on one XCD and share its L2 (identity on the
        // tail of < 32 blocks)
        const long b = blockIdx.x, nb = gridDim.x, main = nb - nb % 32;
        long slot = b;
        if (b < main) {
            const long x = b & 7, j = b >> 3;
            slot = 4 * (((j >> 2) << 3) + x) + (j & 3);
        }
        const long s0 = slot & ~3L;
        const int pos = (int)(slot & 3);
        pw_load_quad_bfly<M, CLP, K, PW_A_INFL>(La, Ta, digA, cbA, topA, s0, pos, l, cbw, t);
        if (pw_late_b(K)) {
            // (an opaque copy of t: the piece offsets and mask bit positions of A's loader are not
            // kept live across A's transform for reuse here)
            auto loadB = [&](u64 (&L)[M], int &T) {
                pw_load_quad_bfly<M, CLP, K, PW_LATE_INFL>(L, T, digB, cbB, topB, s0, pos, l, cbw, pw_launder(t));
            };
            pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp, loadB);
        } else {
            pw_load_quad_bfly<M, CLP, K>(Lb, Tb, digB, cbB, topB, s0, pos, l, cbw, t);
            pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp);
        }
        pw_slot_output<M, LK>(X, TT, H, digC + (size_t)slot * l, cbC + (size_t)slot * cbw, topC + slot, l, t);
    } else {
        // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs (blockIdx mod 8), each
        // with its own L2.  Blocks b and b + 8 take the two slots of one pair, so the second
        // reads of a pair's four inputs hit the same L2 (identity on the tail of < 16 blocks).
        const long b = blockIdx.x, nb = gridDim.x, main = nb - nb % 16;
        long slot = b;
        if (b < main) {
            const long x = b & 7, j = b >> 3;
            slot = 2 * (((j >> 1) << 3) + x) + (j & 1);
        }
        pw_load_pair_bfly<M, CLP>(La, Ta, digA, cbA, topA, slot & ~1L, l, cbw, t, slot & 1);
        if (pw_late_b(K)) {
            auto loadB = [&](u64 (&L)[M], int &T) {
                pw_load_pair_bfly<M, CLP>(L, T, digB, cbB, topB, slot & ~1L, l, cbw, t, slot & 1);
            };
            pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp, loadB);
        } else {
            pw_load_pair_bfly<M, CLP>(Lb, Tb, digB, cbB, topB, slot & ~1L, l, cbw, t, slot & 1);
            pw_slot_product<M, LK>(La, Ta, Lb, Tb, X, Xw, TT, PP, t, stamp);
        }
        pw_slot_output<M, LK>(X, TT, H, digC + (size_t)slot * l, cbC + (size_t)slot * cbw, topC + slot, l, t);
    }
    if (stamp) {
        __syncthreads();
        if (threadIdx.x == 0) stamp[7] = __builtin_amdgcn_s_memtime();
    }
}
