// rkernels.hpp -- register-resident radix-2^LOGG passes for big coefficients
// (l = 1024 PP limbs, PP = 1, 2, 4: the 10^9..10^10-bit configs C2-C4).
//
// Same work and HBM format as k_bpass (bkernels.hpp): one workgroup runs LOGG radix-2
// levels of FFT_radix2_twiddle / FFT_radix2 / IFFT_radix2(_twiddle) (mul_fft.c:1397,
// :786, :1444, :1964) on a butterfly group of G = 2^LOGG coefficients of one column or
// row, with the MFA twiddles (README:89), the fused split (FFT_split_bits, :115) and
// the fused 2^-(depth+1) scaling (:3256-3260).
//
// Why a second big-coefficient kernel: k_bpass keeps the group in LDS (G = 8 at
// l = 2048 fills 147 KB), so one workgroup owns a CU and its HBM load, level and store
// phases run back to back -- the stamps (MPFFT_BP_STAMPS) showed half of every group's
// time waiting on the load.  Here the group lives in VGPRs: 512 threads, thread t owns
// limb pairs pp = t + 512 r (r < PP) of every coefficient, 32 limbs per thread at most
// (G PP <= 16), and LDS is only the exchange buffer for the rotations (<= 78 KB).  Two
// workgroups share a CU, so one's loads and stores overlap the other's levels.
//
// Register form of a residue mod p = 2^N + 1: per limb pair (2q, 2q+1) two limbs and a
// signed overflow count,  x = sum_q (a_q + b_q 2^64 + h_q 2^128) 2^(128 q)  (mod p).
// A butterfly is a 128-bit add/sub per pair (the h absorb the carries, no chain across
// pairs).  Multiplications by 2^e are deferred as in k_bpass (pending exponents, closed
// forms of the slot index); for every pass this kernel takes, a level's relative
// exponent is a whole number of limb *pairs* (host: rho % 128 == 0), so the partner is
// read from LDS by a pair-index shift with a sign flip past 2^N.  The two exponents that
// are not (the MFA twiddle before the row DIF, the inverse twiddle / scaling after the
// row or column DIT) are applied once, by a general rotation through LDS on 32-bit
// digits (rp_rot_all), right after the load or after the last level.
//
// HBM store: reduced form (limbs + carry masks, coeff.hpp): the pair overflow h_q is the
// carry into limb 2q+2, one LDS exchange hands it to the thread owning that limb.
#pragma once
#include "bkernels.hpp"
#include "rdispatch.hpp"

typedef unsigned long long rp_v2u __attribute__((ext_vector_type(2)));

// compiler-only barrier (IR memory order + machine scheduling): keeps LDS reads and the
// arithmetic on them from being hoisted or interleaved en masse (each hoisted value holds
// VGPRs or a 64-bit carry mask in SGPRs; the coefficients already take 80 of the 128 VGPRs)
#define RP_FENCE() do { asm volatile("" ::: "memory"); __builtin_amdgcn_sched_barrier(0); } while (0)

__device__ __forceinline__ u32 rp_uniform(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }

// an opaque copy of the thread index: addresses derived from it in one phase are not
// CSE'd with (and kept live from) another phase -- recomputing them is a few VALU ops,
// keeping them costs the VGPRs the coefficients need
__device__ __forceinline__ int rp_launder(int t)
{
    asm volatile("" : "+v"(t));
    return t;
}

typedef unsigned int rp_v4u __attribute__((ext_vector_type(4)));

struct Pr {
    u32 w[4];   // limbs 2q, 2q+1 as 32-bit words (no 64-bit register-pair constraints)
    int h;      // overflow: weight 2^128 (into limb 2q+2; the last pair's weighs 2^N == -1)
};

__device__ __forceinline__ Pr pr_make(rp_v4u v, int h)
{
    Pr r;
    r.w[0] = v.x;
    r.w[1] = v.y;
    r.w[2] = v.z;
    r.w[3] = v.w;
    r.h = h;
    return r;
}
__device__ __forceinline__ rp_v4u pr_words(const Pr &x) { return rp_v4u{x.w[0], x.w[1], x.w[2], x.w[3]}; }

// 128-bit + overflow arithmetic as 32-bit add/sub-with-carry chains (v_add_co/v_addc:
// five VALU ops per add; the overflow builtins on u64 cost compares and selects instead)
__device__ __forceinline__ u32 lo32(u64 v) { return (u32)v; }
__device__ __forceinline__ u32 hi32(u64 v) { return (u32)(v >> 32); }
__device__ __forceinline__ u64 mk64(u32 lo, u32 hi) { return ((u64)hi << 32) | lo; }

// x + (y ^ m) + cin  (m = 0 or ~0: with cin = 1 that is x - y)
__device__ __forceinline__ Pr pr_addx(const Pr &x, const Pr &y, u32 m, u32 cin)
{
    u32 c;
    Pr r;
    r.w[0] = __builtin_addc(x.w[0], y.w[0] ^ m, cin, &c);
    r.w[1] = __builtin_addc(x.w[1], y.w[1] ^ m, c, &c);
    r.w[2] = __builtin_addc(x.w[2], y.w[2] ^ m, c, &c);
    r.w[3] = __builtin_addc(x.w[3], y.w[3] ^ m, c, &c);
    r.h = (int)__builtin_addc((u32)x.h, (u32)y.h ^ m, c, &c);
    return r;
}

__device__ __forceinline__ Pr pr_add(const Pr &x, const Pr &y) { return pr_addx(x, y, 0u, 0u); }
__device__ __forceinline__ Pr pr_sub(const Pr &x, const Pr &y) { return pr_addx(x, y, ~0u, 1u); }

// (x + s y, x - s y), s = -1 when neg: x + (y ^ m) + neg and x + (y ^ ~m) + !neg
__device__ __forceinline__ void pr_bfly(Pr &u, Pr &v, const Pr &x, const Pr &y, bool neg)
{
    const u32 m = neg ? ~0u : 0u;
    const Pr p = pr_addx(x, y, m, (u32)neg), q = pr_addx(x, y, ~m, (u32)!neg);
    u = p;
    v = q;
}

// branch-free (the sign varies per lane): -x = ~x + 1 over the words and the overflow
__device__ __forceinline__ Pr pr_cneg(const Pr &x, bool neg)
{
    const Pr z = {{0, 0, 0, 0}, 0};
    const u32 m = neg ? ~0u : 0u;
    return pr_addx(z, x, m, (u32)neg);
}

// (lo, hi) += sext(d) for a small signed d, in place; cout = the carry out in {-1, 0, 1}
__device__ __forceinline__ void add_small(u32 &lo, u32 &hi, int d, int &cout)
{
    u32 c;
    lo = __builtin_addc(lo, (u32)d, 0u, &c);
    hi = __builtin_addc(hi, d < 0 ? ~0u : 0u, c, &c);
    cout = (int)c - (d < 0 ? 1 : 0);
}

// exchange slot j: limbs (8 l bytes) then pair overflows (l/2 int16)
template <int PP>
struct RX {
    static constexpr int l = 1024 * PP;
    static constexpr size_t SB = (size_t)9 * l;
    unsigned char *base;
    __device__ __forceinline__ u64 *f(int j) const { return (u64 *)(base + (size_t)j * SB); }
    __device__ __forceinline__ short *h(int j) const { return (short *)(base + (size_t)j * SB + 8 * (size_t)l); }
};

template <int PP, int NT = RP_NT>
__device__ __forceinline__ void rp_pub(const RX<PP> &X, int j, const Pr (&x)[rp_r(PP, NT)], int t)
{
#pragma unroll
    for (int r = 0; r < rp_r(PP, NT); ++r) {
        const int pp = t + NT * r;
        *(rp_v4u *)(X.f(j) + 2 * pp) = pr_words(x[r]);
        X.h(j)[pp] = (short)x[r].h;
    }
}

// pair pp of 2^e y, y published in slot j; e a multiple of 128 bits (whole pairs), e < 2N.
// Returns the pair unsigned; neg = its sign.
template <int PP>
__device__ __forceinline__ Pr rp_get_al(const RX<PP> &X, int j, int pp, u32 e, u32 N, bool &neg)
{
    constexpr int HP = RX<PP>::l / 2;
    const bool sg = e >= N;
    const int Yp = (int)((sg ? e - N : e) >> 7);
    int src = pp - Yp;
    const bool wr = src < 0;
    src += wr ? HP : 0;
    const Pr r = pr_make(*(const rp_v4u *)(X.f(j) + 2 * src), X.h(j)[src]);
    neg = wr != sg;
    return r;
}

// pair pp of 2^e y for any e < 2N (32-bit digit rotation, as bp_ld).  The 5 source digits
// 4pp - y - 1 .. 4pp + 3 - y lie in 3 consecutive limbs m0 .. m0+2 (wrapped ones negated,
// 2^N == -1); the low digit of an even limb 2q+2 also carries the overflow of pair q
// (limb 0: minus the last pair's).  m0's parity depends on y only (workgroup-uniform).
template <int PP>
__device__ __forceinline__ Pr rp_get_gen(const RX<PP> &X, int j, int pp, u32 e, u32 N)
{
    constexpr int l = RX<PP>::l;
    const bool sg = e >= N;
    if (sg) e -= N;
    const int y = (int)(e >> 5), sb = (int)(e & 31);
    const int u0 = 4 * pp - y - 1;     // >= -2l
    const int m0 = u0 >> 1, odd = u0 & 1;
    const u64 *F = X.f(j);
    const short *H = X.h(j);
    i64 seq[6];
    bool swr[3];   // wrap flag per limb: applies to each part *after* the sub-digit split (as bp_ld)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int m = m0 + k;
        const bool wr = m < 0;
        m += wr ? l : 0;
        const u64 f = F[m];
        i64 lo = (i64)(u32)f;
        if (!((m0 + k) & 1)) {         // uniform: even limb, takes a pair overflow
            const i64 hv = H[m ? (m >> 1) - 1 : l / 2 - 1];
            lo += m ? hv : -hv;
        }
        seq[2 * k] = lo;
        seq[2 * k + 1] = (i64)(f >> 32);
        swr[k] = wr;
    }
    i64 o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // source digits D[k+1], D[k] = seq[odd + k + 1], seq[odd + k] (selects: odd is uniform,
        // and a runtime index would put seq in scratch)
        const i64 d1 = odd ? seq[k + 2] : seq[k + 1], d0 = odd ? seq[k + 1] : seq[k];
        const bool w1 = odd ? swr[(k + 2) >> 1] : swr[(k + 1) >> 1], w0 = odd ? swr[(k + 1) >> 1] : swr[k >> 1];
        o[k] = bp_cneg(bp_lo(d1, sb), w1) + bp_cneg(bp_hi(d0, sb), w0);
    }
    if (sg) {
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = -o[k];
    }
    const i128 t0 = (i128)o[0] + ((i128)o[1] << 32);
    const i128 t1 = (i128)o[2] + ((i128)o[3] << 32) + (t0 >> 64);
    Pr r;
    r.w[0] = (u32)t0;
    r.w[1] = (u32)((u64)t0 >> 32);
    r.w[2] = (u32)t1;
    r.w[3] = (u32)((u64)t1 >> 32);
    r.h = (int)(i64)(t1 >> 64);
    return r;
}

// pair pp of 2^e y for any e < 2N (the general rotation), from two aligned reads: with
// e = ea + d (ea whole pairs, d < 128 bits), z = 2^ea y has signed pairs z_q = w_q + h_q 2^128
// (rp_get_al, signs folded), and 2^d z_q = lo(z_q) + hi(z_q) 2^128 with
// lo(z_q) = (w_q << d) mod 2^128, hi(z_q) = floor(z_q / 2^(128 - d)), so
//   pair pp of 2^d z = lo(z_pp) + hi(z_(pp-1)),   pair 0: lo(z_0) - hi(z_(HP-1))  (2^N = -1;
// the negation after the floor, not before).  Checked against exact arithmetic by a Python
// model of the same decomposition (k_rpass).
// d = 32 B + s with B, s workgroup-uniform: word selects resolve at compile time (rp_shift_pair<B>)
// and every bit shift is one v_alignbit -- about a third of rp_get_gen's 64-bit digit arithmetic.
__device__ __forceinline__ u32 rp_fun(u32 hi, u32 lo, u32 s) { return s ? __builtin_amdgcn_alignbit(hi, lo, 32 - s) : hi; }

template <int B>
__device__ __forceinline__ Pr rp_shift_pair(const Pr &a, const Pr &b, u32 s, bool sub)
{
    const u32 bs = b.h < 0 ? ~0u : 0u;
    auto aw = [&](int i) -> u32 { return i >= 0 && i < 4 ? a.w[i] : 0u; };            // i compile-time
    auto bw = [&](int i) -> u32 { return i < 4 ? b.w[i] : i == 4 ? (u32)b.h : bs; };    // i >= 0 compile-time
    Pr lo, hi;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lo.w[k] = rp_fun(aw(k - B), aw(k - B - 1), s);        // bits [32k, 32k + 32) of w_pp << d
        hi.w[k] = rp_fun(bw(k + 4 - B), bw(k + 3 - B), s);    // bits [32k, ..) of floor(z_(pp-1) / 2^(128 - d))
    }
    lo.h = 0;
    hi.h = (int)rp_fun(bw(8 - B), bw(7 - B), s);              // its signed part above 2^128
    const u32 m = sub ? ~0u : 0u;
    return pr_addx(lo, hi, m, (u32)sub);
}

template <int PP>
__device__ __forceinline__ Pr rp_get_rot(const RX<PP> &X, int j, int pp, u32 e, u32 N)
{
    constexpr int HP = RX<PP>::l / 2;
    const u32 d = e & 127;
    bool n0, n1;
    const Pr a = pr_cneg(rp_get_al<PP>(X, j, pp, e - d, N, n0), n0);
    if (d == 0) return a;   // workgroup-uniform
    const Pr b = pr_cneg(rp_get_al<PP>(X, j, pp ? pp - 1 : HP - 1, e - d, N, n1), n1);
    const u32 s = d & 31;
    const bool wrap = pp == 0;
    switch (d >> 5) {       // workgroup-uniform
    case 0: return rp_shift_pair<0>(a, b, s, wrap);
    case 1: return rp_shift_pair<1>(a, b, s, wrap);
    case 2: return rp_shift_pair<2>(a, b, s, wrap);
    default: return rp_shift_pair<3>(a, b, s, wrap);
    }
}

// The bit part of a general rotation on values already rotated by whole pairs (rotated
// load): pair pp of 2^d z = lo(z_pp) + hi(z_(pp-1)) (pair 0: minus hi(z_(HP-1))), as rp_get_rot,
// with z_(pp-1) taken from the register of lane - 1 (DPP wave_ror:1) -- no publish of the
// coefficients.  Lane 0 of each wave needs lane 63 of the wave below (pair pp - 1 = thread
// t - 1; thread 0 of round r: thread NT - 1 of round r - 1, round 0: pair HP - 1): those
// lanes' pairs go through a small LDS table EDGE (NT/64 x G x R x 5 words), one barrier.
// d = e mod 128 = 32 B + s, workgroup-uniform per slot.
#ifndef RP_GX_LOAD
#define RP_GX_LOAD 1   // 0: the round-3 form (plain load, general rotation through LDS), A/B builds only
#endif
#ifndef RP_SPLIT_ZSKIP
#define RP_SPLIT_ZSKIP 1   // 0 (A/B builds): the split pass exchanges its zero slots like any other
#endif
#ifndef RP_SPLIT_LDS
#define RP_SPLIT_LDS 1     // 0 (A/B builds): the split pass's per-slot guarded loads for whole operands too
#endif
#ifndef RP_SPLIT_PROBE
#define RP_SPLIT_PROBE 0   // 1: timing probe, the split pass's source loads replaced by arithmetic (A/B builds only)
#endif
__device__ __forceinline__ u32 rp_ror1(u32 v) { return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xF, 0xF, false); }

template <int G, int PP, int NT, typename EF>
__device__ __forceinline__ void rp_shift_all(Pr (&x)[G][rp_r(PP, NT)], u32 *EDGE, EF ef, int t)
{
    constexpr int R = rp_r(PP, NT), NW = NT / 64;
    const int lane = t & 63, wv = t >> 6;
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < G; ++i)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                u32 *q = EDGE + 5 * ((wv * G + i) * R + r);
                q[0] = x[i][r].w[0];
                q[1] = x[i][r].w[1];
                q[2] = x[i][r].w[2];
                q[3] = x[i][r].w[3];
                q[4] = (u32)x[i][r].h;
            }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const u32 d = ef(i) & 127;
        if (d == 0) continue;   // workgroup-uniform
        const u32 s = d & 31;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            RP_FENCE();
            Pr b;
            b.w[0] = rp_ror1(x[i][r].w[0]);
            b.w[1] = rp_ror1(x[i][r].w[1]);
            b.w[2] = rp_ror1(x[i][r].w[2]);
            b.w[3] = rp_ror1(x[i][r].w[3]);
            b.h = (int)rp_ror1((u32)x[i][r].h);
            if (lane == 0) {
                const int w2 = wv ? wv - 1 : NW - 1, r2 = wv ? r : (r ? r - 1 : R - 1);
                const u32 *q = EDGE + 5 * ((w2 * G + i) * R + r2);
                b.w[0] = q[0];
                b.w[1] = q[1];
                b.w[2] = q[2];
                b.w[3] = q[3];
                b.h = (int)q[4];
            }
            const bool wrap = t == 0 && r == 0;   // pair 0: minus hi(z_(HP-1))
            switch (d >> 5) {   // workgroup-uniform
            case 0: x[i][r] = rp_shift_pair<0>(x[i][r], b, s, wrap); break;
            case 1: x[i][r] = rp_shift_pair<1>(x[i][r], b, s, wrap); break;
            case 2: x[i][r] = rp_shift_pair<2>(x[i][r], b, s, wrap); break;
            default: x[i][r] = rp_shift_pair<3>(x[i][r], b, s, wrap); break;
            }
        }
    }
}

// Exponents in 32 bits: every one is reduced mod 2N < 2^20 (l <= 4096), and a level
// twiddle (k_pass :212-229) is below N (SGPR pressure: the 64-bit forms spilled).
__device__ __forceinline__ u32 rp_mod2n(u32 e, u32 N2)
{
    e = e >= 2 * N2 ? e - 2 * N2 : e;
    return e >= N2 ? e - N2 : e;
}

// level twiddle of the pair whose upper element is k at level index li (bp_tw in 32 bits)
template <int LOGG, int DIR>
__device__ __forceinline__ u32 rp_tw(const PassArgs &a, const BGeo &g, int li, int k)
{
    const int JB = DIR == 0 ? LOGG - 1 - li : li;
    const int level = DIR == 0 ? a.lvl0 + li : a.lvl0 + LOGG - 1 - li;
    const u32 h = 1u << (a.lbM - level - 1);
    const u32 unit = (u32)a.rho << level;
    return (u32)(g.pos0 & (h - 1)) * unit + (u32)(k & ((1 << JB) - 1)) * (u32)g.pstep * unit;
}

// DIF pending exponent of position p after levels [lo, hi) of a length-2^lbM transform with
// root 2^rho (in-place DIF: the bottom element of a level-lev butterfly takes the top one's
// pending exponent plus the twiddle rho 2^lev (p mod h); the later levels' bits are the top's,
// so every term is rho 2^lev (p mod 2^(lbM - hi)) -- each below N)
__device__ __forceinline__ u32 rp_pend_pos(u32 rho, int lbM, int lo, int hi, u32 p, u32 N2)
{
    const u32 xm = p & ((1u << (lbM - hi)) - 1);
    u32 e = 0;
    for (int lev = lo; lev < hi; ++lev)
        if ((p >> (lbM - lev - 1)) & 1) e = rp_mod2n(e + (rho << lev) * xm, N2);
    return e;
}

// DIF pending exponent of slot s after `done` levels of this pass, including the levels an
// earlier pass left pending (pcarry; bp_pend without the MFA twiddle term: rp applies that on load)
template <int LOGG>
__device__ __forceinline__ u32 rp_pend(const PassArgs &a, const BGeo &g, int done, int s, u32 N2)
{
    return rp_pend_pos((u32)a.rho, a.lbM, a.lvl0 - a.pcarry, a.lvl0 + done, (u32)(g.pos0 + s * g.pstep), N2);
}

// x_i <- 2^E(i) x_i for all G slots (general exponents), NX slots per LDS round
template <int G, int PP, int NX, int NT = RP_NT, typename EF>
__device__ __forceinline__ void rp_rot_all(Pr (&x)[G][rp_r(PP, NT)], const RX<PP> &X, EF efn, u32 N, int t)
{
    t = rp_launder(t);
#pragma unroll
    for (int i0 = 0; i0 < G; i0 += NX) {
#pragma unroll
        for (int q = 0; q < NX && i0 + q < G; ++q) rp_pub<PP, NT>(X, q, x[i0 + q], t);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NX && i0 + q < G; ++q) {
            const u32 e = efn(i0 + q);
            if (e == 0) continue;   // workgroup-uniform
#pragma unroll
            for (int r = 0; r < rp_r(PP, NT); ++r) {
                RP_FENCE();   // one pair position at a time (VGPRs)
                x[i0 + q][r] = rp_get_rot<PP>(X, q, t + NT * r, e, N);
            }
        }
        __syncthreads();
    }
}

// Every exponent a pass needs, as a table one workgroup computes once in LDS (lane e
// computes entry e): the kernel then reads them back as uniform values instead of
// keeping dozens of scalar products live (they spilled).  Layout: [0, G) the general
// multipliers (MFA twiddle before a DIF pass, bp_post after a DIT pass); [G, 2G) the
// pending exponent of each slot after the last DIF level (applied by one aligned
// rotation round); then G/2 partner exponents per level at 2G + li G/2.
template <int LOGG, int DIR, bool GX, bool CIN = false>
__device__ __forceinline__ u32 rp_exp_entry(const PassArgs &a0, const BGeo &g, int e, u32 N2, u32 cadd)
{
    constexpr int G = 1 << LOGG;
    // CIN: the inputs owe the pending exponents of levels [lvl0 - pcarry, lvl0); entries [0, G)
    // hold them (applied by the rotated load), and the pass then owes only its own levels
    PassArgs a = a0;
    if (CIN) a.pcarry = 0;
    if (e < G) {
        if (CIN) return rp_pend_pos((u32)a0.rho, a0.lbM, a0.lvl0 - a0.pcarry, a0.lvl0, (u32)(g.pos0 + e * g.pstep), N2);
        if (DIR == 1 && a.tw_mode == 3) {   // the inverse MFA twiddle (and the scaling) on load, rows of a column block
            const long row = (long)a.pos_off + g.pos0 + (long)e * g.pstep;
            const u64 t = bp_mod2n(g.tw0 * (u64)revbin_dev(row, a.tw_lbR), N2);
            return (u32)bp_mod2n((t ? N2 - t : 0) + a.scale_e, N2);
        }
        if (!GX) return 0;
        return DIR == 0 ? (u32)bp_mod2n(g.tw0 + (u64)e * g.twst + cadd, N2) : (u32)bp_post(a, g, e, N2);
    }
    if (e < 2 * G) return DIR == 0 ? rp_pend<LOGG>(a, g, LOGG, e - G, N2) : 0;
    e -= 2 * G;
    const int li = e / (G / 2), r = e % (G / 2);
    if (li >= LOGG) return 0;
    const int JB = DIR == 0 ? LOGG - 1 - li : li;
    const int i = ((r >> JB) << (JB + 1)) | (r & ((1 << JB) - 1)), k = i | (1 << JB);
    if (DIR == 0) {
        const u32 Pi = rp_pend<LOGG>(a, g, li, i, N2), Pk = rp_pend<LOGG>(a, g, li, k, N2);
        return Pk >= Pi ? Pk - Pi : Pk + N2 - Pi;
    }
    const u32 tw = rp_mod2n(rp_tw<LOGG, 1>(a, g, li, k), N2);
    return tw ? N2 - tw : 0;
}



// x_i <- 2^E(i) x_i for all G slots, every E a whole number of limb pairs
template <int G, int PP, int NX, int NT = RP_NT, typename EF>
__device__ __forceinline__ void rp_rot_all_al(Pr (&x)[G][rp_r(PP, NT)], const RX<PP> &X, EF efn, u32 N, int t)
{
    t = rp_launder(t);
#pragma unroll
    for (int i0 = 0; i0 < G; i0 += NX) {
#pragma unroll
        for (int q = 0; q < NX && i0 + q < G; ++q)
            if (efn(i0 + q)) rp_pub<PP, NT>(X, q, x[i0 + q], t);   // uniform: slot 0 (e = 0) stays put
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NX && i0 + q < G; ++q) {
            const u32 e = efn(i0 + q);
            if (e == 0) continue;
#pragma unroll
            for (int r = 0; r < rp_r(PP, NT); ++r) {
                RP_FENCE();
                bool ng;
                const Pr y = rp_get_al<PP>(X, q, t + NT * r, e, N, ng);
                x[i0 + q][r] = pr_cneg(y, ng);
            }
        }
        __syncthreads();
    }
}

// ---- HBM <-> register pairs (k_rpass, k_rpair) ------------------------------------
// Carry masks -> one 16-bit code per limb pair in LDS (low byte: carry out of limb 2pp,
// high byte: carry out of limb 2pp+1, plus the carry limb for the last pair); one thread
// per (slot, 64-limb row) of the first NS slots, slot i's index at SL[i] (LDS).
// Staged in two halves, so a kernel can issue its limb loads between them: the
// mask (and carry-limb) loads go out first, the limb loads behind them, and the code
// computation then waits only for the masks (in-order vmcnt) while the limbs are in flight.
// (staging the codes before the limb loads serialised two HBM round trips: the limb loads'
// slot indices come from LDS, read after the code stores, which wait for the masks.)
struct RpCodes {
    rp_v2u pn;
    int tv;
};

template <int NS, int PP>
__device__ __forceinline__ RpCodes rp_codes_load(const Coef &st, const u32 *SL, int t)
{
    constexpr int l = 1024 * PP, cbw = 2 * l / 64, rows = l / 64;
    RpCodes c{rp_v2u{0, 0}, 0};
    if (t >= NS * rows) return c;
    const int i = t / rows, W = t % rows;
    const long sl = (long)SL[i];
    c.pn = *(const rp_v2u *)(st.cb + (size_t)sl * cbw + 2 * W);
    c.tv = W == rows - 1 ? st.top[sl] : 0;
    return c;
}

template <int NS, int PP>
__device__ __forceinline__ void rp_codes_store(unsigned short *CODE, const RpCodes &cd, int t)
{
    constexpr int l = 1024 * PP, HP = l / 2, rows = l / 64;
    if (t >= NS * rows) return;
    const int i = t / rows, W = t % rows;
    const rp_v2u pn = cd.pn;
    rp_v2u *dst = (rp_v2u *)(CODE + i * HP + 32 * W);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        u64 w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            u64 acc = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 8 * c + 4 * h + k, b = 2 * j;
                const int c0 = (int)((pn.x >> b) & 1) - (int)((pn.y >> b) & 1);
                int c1 = (int)((pn.x >> (b + 1)) & 1) - (int)((pn.y >> (b + 1)) & 1);
                c1 += j == 31 ? cd.tv : 0;
                acc |= (u64)((c0 & 0xff) | ((c1 & 0xff) << 8)) << (16 * k);
            }
            w[h] = acc;
        }
        dst[c] = rp_v2u{w[0], w[1]};
    }
}

// bit j of the wave-uniform x -> bit 2j: s_bitreplicate doubles every bit, the mask keeps one
__device__ __forceinline__ u64 rp_spread32(u32 x)
{
    u64 v;
    asm("s_bitreplicate_b64_b32 %0, %1" : "=s"(v) : "s"(x));
    return v & 0x5555555555555555ull;
}

// limbs of the first NS slots (slot i at the uniform index SL[i])
template <int NS, int NSX, int PP, int NT = RP_NT>
__device__ __forceinline__ void rp_load_limbs(Pr (&x)[NSX][rp_r(PP, NT)], const Coef &st, const u32 *SL, int t)
{
    constexpr int l = 1024 * PP;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const long sl = (long)rp_uniform(SL[i]);
#pragma unroll
        for (int r = 0; r < rp_r(PP, NT); ++r)
            x[i][r] = pr_make(*(const rp_v4u *)(st.dig + (size_t)sl * l + 2 * (t + NT * r)), 0);
    }
}

// codes -> pair form: limb 2pp's carry moves into limb 2pp+1, limb 2pp+1's (and the carry
// limb) is the pair overflow h.  Ends with a barrier: CODE aliases the exchange slots.
// Rotated load (k_rpass MODE 3): slot i is read already multiplied by 2^E_i, E_i a whole
// number of limb pairs (< 2N, workgroup-uniform): pair pp of 2^E y is pair pp - Y of y
// (Y = (E mod N) / 128), negated when that index wraps below 0 (2^N == -1) xor E >= N.  The
// pair's code (its carries) travels with it; its overflow h keeps meaning "into the next
// pair" in the rotated frame, including across the wrap (the negated top pair lands at Y - 1
// and its overflow at Y, which is where -h 2^N times 2^(128 Y) belongs).  So the pending
// exponents an earlier pass left behind cost no LDS round: addresses and one negation.
__device__ __forceinline__ int rp_rot_src(int pp, u32 e, u32 N, int HP, bool &neg)
{
    const bool sg = e >= N;
    int src = pp - (int)((sg ? e - N : e) >> 7);
    const bool wr = src < 0;
    src += wr ? HP : 0;
    neg = wr != sg;
    return src;
}

template <int NS, int NSX, int PP, int NT, typename EF>
__device__ __forceinline__ void rp_load_limbs_rot(Pr (&x)[NSX][rp_r(PP, NT)], const Coef &st, const u32 *SL, EF ef,
                                                  int t)
{
    constexpr int l = 1024 * PP, HP = l / 2;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const long sl = (long)rp_uniform(SL[i]);
        const u32 e = ef(i);
#pragma unroll
        for (int r = 0; r < rp_r(PP, NT); ++r) {
            bool ng;
            const int src = rp_rot_src(t + NT * r, e, (u32)(64 * l), HP, ng);
            x[i][r] = pr_make(*(const rp_v4u *)(st.dig + (size_t)sl * l + 2 * src), 0);
        }
        RP_FENCE();   // a slot's addresses die with its loads (all loads stay in flight)
    }
}

template <int NS, int NSX, int PP, int NT, typename EF>
__device__ __forceinline__ void rp_decode_rot(Pr (&x)[NSX][rp_r(PP, NT)], const unsigned short *CODE, EF ef, int t)
{
    constexpr int HP = 512 * PP;
    t = rp_launder(t);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const u32 e = ef(i);
#pragma unroll
        for (int r = 0; r < rp_r(PP, NT); ++r) {
            RP_FENCE();
            bool ng;
            const int src = rp_rot_src(t + NT * r, e, (u32)(128 * HP), HP, ng);
            const int code = CODE[i * HP + src];
            const int c0 = (signed char)(code & 0xff), c1 = (signed char)(code >> 8);
            int cc;
            add_small(x[i][r].w[2], x[i][r].w[3], c0, cc);
            x[i][r].h = c1 + cc;
            x[i][r] = pr_cneg(x[i][r], ng);
        }
    }
    __syncthreads();
}

template <int NS, int NSX, int PP, int NT = RP_NT>
__device__ __forceinline__ void rp_decode(Pr (&x)[NSX][rp_r(PP, NT)], const unsigned short *CODE, int t)
{
    constexpr int HP = 512 * PP;
    t = rp_launder(t);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
#pragma unroll
        for (int r = 0; r < rp_r(PP, NT); ++r) {
            RP_FENCE();   // one code read at a time (else all are hoisted: VGPRs)
            const int code = CODE[i * HP + t + NT * r];
            const int c0 = (signed char)(code & 0xff), c1 = (signed char)(code >> 8);
            int cc;   // b += c0 (branch-free: divergent branches here cost the allocator dearly)
            add_small(x[i][r].w[2], x[i][r].w[3], c0, cc);
            x[i][r].h = c1 + cc;
        }
    }
    __syncthreads();
}

// store (reduced form) of the slots i < NS with keep(i): pair overflows -> LDS (HX, over the
// exchange slots: callers end their last LDS phase with a barrier), then limb 2pp takes the
// overflow of pair pp - 1 (pair 0: minus the last pair's, 2^N == -1); its carry out goes
// into the masks, limb 2pp+1 carries 0
template <int NS, int NSX, int PP, int NT = RP_NT, typename KEEP>
__device__ __forceinline__ void rp_store(const Pr (&x)[NSX][rp_r(PP, NT)], const Coef &st, const u32 *SL, KEEP keep, short *HX, int t)
{
    constexpr int l = 1024 * PP, HP = l / 2, cbw = 2 * l / 64, R = rp_r(PP, NT);
    t = rp_launder(t);
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int r = 0; r < R; ++r) HX[i * HP + t + NT * r] = (short)x[i][r].h;
    __syncthreads();
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if (!keep(i)) continue;   // workgroup-uniform
        const long sl = (long)rp_uniform(SL[i]);
        u64 *dst = st.dig + (size_t)sl * l;
        u64 *cbp = st.cb + (size_t)sl * cbw;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            RP_FENCE();
            const int pp = t + NT * r;
            const int hv = HX[i * HP + (pp ? pp - 1 : HP - 1)];
            const int hin = pp ? hv : -hv;
            int k0;
            u32 w0 = x[i][r].w[0], w1 = x[i][r].w[1];   // x itself stays intact (k_rpass FILL stores it twice)
            add_small(w0, w1, hin, k0);
            *(rp_v4u *)(dst + 2 * pp) = rp_v4u{w0, w1, x[i][r].w[2], x[i][r].w[3]};
            // mask words of rows 2 (wv + NW r) (NW = NT / 64 waves; pairs of lanes 0..31) and +1
            // (lanes 32..63): bit 2j is pair j's even limb (odd limbs carry nothing) -- one ballot
            // per sign, each half spread to the even bits by s_bitreplicate (no lane shuffles; a
            // shift-and-mask spread on the scalar unit measured slower than the shuffles)
            const u64 bp = __ballot(k0 == 1), bn = __ballot(k0 == -1);
            const u64 pa = rp_spread32((u32)bp), na = rp_spread32((u32)bn);
            const u64 pb = rp_spread32((u32)(bp >> 32)), nb = rp_spread32((u32)(bn >> 32));
            if (lane < 2)
                *(rp_v2u *)(cbp + 2 * (2 * (wv + (NT / 64) * r) + lane)) = lane ? rp_v2u{pb, nb} : rp_v2u{pa, na};
        }
        if (t == 0) st.top[sl] = 0;
    }
}

// every coefficient word materialised in a register at this point, and a scheduling fence: the
// DIT kernels otherwise interleave the last level's butterflies with what follows (the store or
// the general rotation) and spill 60-130 B; this boundary removes that
template <int G, int R>
__device__ __forceinline__ void rp_pin(Pr (&x)[G][R])
{
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
        for (int r = 0; r < R; ++r)
            asm volatile("" : "+v"(x[i][r].w[0]), "+v"(x[i][r].w[1]), "+v"(x[i][r].w[2]), "+v"(x[i][r].w[3]), "+v"(x[i][r].h));
    RP_FENCE();
}

// MODE: DIR 0: 0 plain, 1 MFA twiddle on load, 2 split on load (first column pass),
//               3 plain with inputs that still owe an earlier pass's pending exponents
//               (PassArgs::pcarry: applied by a rotated load, rp_load_limbs_rot, so the
//               first level still runs in registers);
//       DIR 1: bit 0 general final multipliers (inverse twiddle / scaling), bit 1 the pass
//               holds the transform's last DIT level (h = 1: its first level needs no rotation),
//               bit 2 the truncated inverse's FILL step (PassArgs::fill_*; not with bit 0),
//               bit 3 the inverse MFA twiddle and the scaling applied on load (PassArgs::tw_mode
//               3: the first pass of a column block, the rows' last pass then plain -- fold plans)
// (compile-time, so the register-only level and the LDS level are never both in one kernel:
// a runtime choice between them spilled)
template <int LOGG, int PP, int DIR, int MODE>
__global__ __launch_bounds__(rp_nt(1024 * PP, LOGG, DIR), 4) void k_rpass(PassArgs a)
{
    constexpr int NT = rp_nt(1024 * PP, LOGG, DIR), R = rp_r(PP, NT);
    constexpr bool GX = DIR == 0 ? MODE == 1 : (MODE & 1) != 0, SPLIT = DIR == 0 && MODE == 2,
                   CIN = DIR == 0 && MODE == 3, HL = DIR == 1 && (MODE & 2) != 0,
                   FILL = DIR == 1 && (MODE & 4) != 0, LTW = DIR == 1 && (MODE & 8) != 0;
    pass_clear_flags(a);
    constexpr int G = 1 << LOGG, NX = G / 2 > 2 ? G / 2 : 2;
    constexpr int l = 1024 * PP, HP = l / 2, cbw = 2 * l / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RX<PP> X{smem};
    const int t = threadIdx.x;
    const u32 N = (u32)a.N, N2 = 2 * (u32)a.N;
    const int op = blockIdx.y;
    Coef st;
    st.dig = a.dig[op];
    st.cb = a.cb[op];
    st.top = a.top[op];
    // group geometry is workgroup-uniform: keep it in SGPRs (readfirstlane), the VGPRs
    // are all needed for the coefficients
    const int sub = __builtin_amdgcn_readfirstlane((int)(blockIdx.x / a.ngroups));
    const int grp = __builtin_amdgcn_readfirstlane((int)(a.grp0 + blockIdx.x % a.ngroups));
    const int lobits = a.lbM - a.lvl0 - LOGG;
    const int lo = grp & ((1 << lobits) - 1);
    const int hi = grp >> lobits;
    const int bstart = hi << (a.lbM - a.lvl0);
    if (DIR == 0 && (bstart >= a.need || bstart + (1 << (a.lbM - a.lvl0)) <= a.need_lo)) return;   // whole block past the truncation point / outside the rows needed (workgroup-uniform)
    BGeo g;
    g.pos0 = bstart | lo;
    g.pstep = 1 << lobits;
    g.sbase = (long)sub * a.sub_stride;
    const u64 rsub = a.tw_mode && a.tw_mode != 3 ? (u64)revbin_dev(a.sub_off + sub, a.tw_lbR) : 0;
    g.tw0 = a.tw_mode == 3 ? a.tw_w * (u64)(a.sub_off + sub) : a.tw_w * (u64)(a.pos_off + g.pos0) * rsub;   // 3: the column
    g.twst = a.tw_w * (u64)g.pstep * rsub;
    auto slot_lane = [&](int i) -> long {   // any i (the code staging has two slots per wave)
        const int ps = a.pos_off + g.pos0 + i * g.pstep;
        return g.sbase + (long)(ps >> a.pbb) * a.pbs + (long)(ps & ((1 << a.pbb) - 1)) * a.pos_stride;
    };
    auto slot_of = [&](int i) -> long { return wv_uniform(slot_lane(i)); };   // i wave-uniform: SGPRs
    // zero inputs (positions >= zero_from) only occur in the split pass (host: rp_usable)
    auto zero_in = [&](int i) -> bool { return SPLIT && g.pos0 + i * g.pstep >= a.zero_from; };
    // exponent table (rp_exp_entry) and the G slot indices: read back as uniform values
    // where needed (kept live from load to store, the 64-bit slot addresses spilled)
    constexpr int NEXP = 2 * G + (G / 2) * LOGG;
    u32 *EXPT = (u32 *)(smem + NX * RX<PP>::SB);
    u32 *SLT = EXPT + NEXP;
    if (t < NEXP) EXPT[t] = rp_exp_entry<LOGG, DIR, GX, CIN>(a, g, t, N2, 0u);
    else if (t < NEXP + G) SLT[t - NEXP] = (u32)slot_lane(t - NEXP);
    __syncthreads();
    const u64 *src = SPLIT ? a.src[op] : nullptr;
    // diagnostics (MPFFT_RP_STAMPS): thread 0 stamps the phase boundaries of this workgroup
    unsigned long long *stamp = a.dbg ? a.dbg + 8 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) : nullptr;
#define RP_STAMP(k) do { if (stamp && t == 0) stamp[k] = __builtin_amdgcn_s_memtime(); } while (0)
    RP_STAMP(0);

    // ---- load ------------------------------------------------------------------------
    unsigned short *CODE = (unsigned short *)smem;   // G HP codes (over the exchange slots)
    Pr x[G][R];
    u32 *EDGE = SLT + G;   // rp_shift_all's lane-63 table (rp_lds)
    if ((DIR == 0 && GX && RP_GX_LOAD) || LTW) {   // MFA twiddle 2^(tw0 + s twst) of slot s (README:89), so every level is pair-aligned:
        // whole pairs by the rotated load, the rest by neighbour pairs in registers
        auto ef = [&](int i) -> u32 { return rp_uniform(EXPT[i]); };
        const RpCodes cd = rp_codes_load<G, PP>(st, SLT, t);
        rp_load_limbs_rot<G, G, PP, NT>(x, st, SLT, ef, t);
        rp_codes_store<G, PP>(CODE, cd, t);
        __syncthreads();
        rp_decode_rot<G, G, PP, NT>(x, CODE, ef, t);
        rp_pin<G, R>(x);
        rp_shift_all<G, PP, NT>(x, EDGE, ef, t);
    } else if (CIN) {   // owed pending exponents: rotated load (EXPT[0, G))
        auto ef = [&](int i) -> u32 { return rp_uniform(EXPT[i]); };
        const RpCodes cd = rp_codes_load<G, PP>(st, SLT, t);
        rp_load_limbs_rot<G, G, PP, NT>(x, st, SLT, ef, t);
        rp_codes_store<G, PP>(CODE, cd, t);
        __syncthreads();
        rp_decode_rot<G, G, PP, NT>(x, CODE, ef, t);
        rp_pin<G, R>(x);   // the rotated values materialised before the register level (else spills)
    } else if (!SPLIT) {
        const RpCodes cd = rp_codes_load<G, PP>(st, SLT, t);   // masks first, limbs behind them
        rp_load_limbs<G, G, PP, NT>(x, st, SLT, t);
        rp_codes_store<G, PP>(CODE, cd, t);
        __syncthreads();
        rp_decode<G, G, PP, NT>(x, CODE, t);
    } else {   // first forward column pass: FFT_split_bits fused into the load
        // pair pp of a split coefficient from the three source limbs q .. q + 2 holding its bits
        auto split_pair = [](u64 x0, u64 x1, u64 x2, int sh, u64 left) -> Pr {
            u64 f0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
            u64 f1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
            f0 = left < 64 ? f0 & ((((u64)1) << left) - 1) : f0;
            f1 = left <= 64 ? 0 : left < 128 ? f1 & ((((u64)1) << (left - 64)) - 1) : f1;
            return pr_make(rp_v4u{(u32)f0, (u32)(f0 >> 32), (u32)f1, (u32)(f1 >> 32)}, 0);
        };
        // staged form (whole operands): every live slot's source span -- bits1 < N/2 bits, so at most
        // l/2 + 2 limbs from the even limb below its first -- read with coalesced 16-B loads by
        // consecutive threads, all slots' loads in flight at once, parked in the exchange slots; each
        // thread then reads its three limbs per pair back from LDS
        constexpr int SWP = l / 4 + 2, SW = 2 * SWP, KR = (G * SWP + NT - 1) / NT;
        constexpr bool STAGE = RP_SPLIT_LDS && (size_t)G * SW * 8 <= (size_t)NX * RX<PP>::SB;
        if (STAGE && !a.src_chunk) {
            u64 *S = (u64 *)smem;
            const long nsv = a.nsrc[op];
            auto slot_q0 = [&](int i) -> long {   // the even source limb staged slot i starts at
                const long j = (long)(a.pos_off + g.pos0 + i * g.pstep) * a.jNC + a.sub_off + sub;
                return (long)(((u64)j * a.bits1) >> 6) & ~1L;
            };
            rp_v4u v[KR];
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                const int idx = t + NT * k, i = idx / SWP, u = idx - i * SWP;
                v[k] = rp_v4u{0, 0, 0, 0};
                if (i < G && !zero_in(i)) {
                    const long q = slot_q0(i) + 2 * u;
                    if (q + 1 < nsv) {
                        v[k] = *(const rp_v4u *)(src + q);
                    } else if (q < nsv) {
                        const u64 w = src[q];
                        v[k] = rp_v4u{(u32)w, (u32)(w >> 32), 0, 0};
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                const int idx = t + NT * k, i = idx / SWP, u = idx - i * SWP;
                if (i < G && !zero_in(i)) *(rp_v4u *)(S + (long)i * SW + 2 * u) = v[k];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const bool z = zero_in(i);
                const long j = (long)(a.pos_off + g.pos0 + i * g.pstep) * a.jNC + a.sub_off + sub;
                const long qa = (long)(((u64)j * a.bits1) >> 6) & ~1L;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int pp = t + NT * r;
                    x[i][r] = Pr{{0, 0, 0, 0}, 0};
                    const u64 left = (u64)pp * 128 < a.bits1 ? a.bits1 - (u64)pp * 128 : 0;
                    if (z || !left) continue;
                    const u64 off = (u64)j * a.bits1 + (u64)pp * 128;
                    const u64 *sp = S + (long)i * SW + ((long)(off >> 6) - qa);
                    x[i][r] = split_pair(sp[0], sp[1], sp[2], (int)(off & 63), left);
                }
            }
            __syncthreads();   // the staging area is the exchange slots level 1 publishes into
        } else {
            // one slot at a time, guarded loads (a zero slot, and the lanes past the coefficient's
            // bits1 bits -- the upper half of every split coefficient -- issue none).  Round 5 put four
            // slots' loads in flight from clamped addresses: C3's pass 0.735 -> 0.885 ms, C4's 5.17 ->
            // 6.05 (every dead lane loaded); with wave-uniform skips of the dead waves and zero slots
            // still 0.771 / 5.29 ms (profiles/r06/split_ab.txt)
#pragma unroll
            for (int i = 0; i < G; ++i) {
                __builtin_amdgcn_sched_barrier(0);   // 3 source limbs per pair, a slot at a time
                const bool z = zero_in(i);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int pp = t + NT * r;
                    x[i][r] = Pr{{0, 0, 0, 0}, 0};
                    if (z) continue;
                    const u64 left = (u64)pp * 128 < a.bits1 ? a.bits1 - (u64)pp * 128 : 0;   // bits of the coefficient here
                    const long j = (long)(a.pos_off + g.pos0 + i * g.pstep) * a.jNC + a.sub_off + sub;
                    const u64 off = (u64)j * a.bits1 + (u64)pp * 128;
                    const long q = (long)(off >> 6);
                    const long ns = left ? a.nsrc[op] : 0;
                    const SrcSlice sv{a.src_chunk, a.jNC, a.sub_off};
#if RP_SPLIT_PROBE   // timing probe (A/B builds only, wrong products): the split pass without its source loads
                    const u64 x0 = left ? (u64)q * 0x9e3779b97f4a7c15ull : 0, x1 = x0 ^ (u64)j, x2 = x1 + 1;
#else
                    const u64 x0 = src_limb(src, ns, sv, j, a.bits1, q), x1 = src_limb(src, ns, sv, j, a.bits1, q + 1),
                              x2 = src_limb(src, ns, sv, j, a.bits1, q + 2);
#endif
                    x[i][r] = split_pair(x0, x1, x2, (int)(off & 63), left);
                }
            }
        }
    }
    RP_STAMP(1);
    if (DIR == 0 && GX && !RP_GX_LOAD) {   // (A/B variant) the MFA twiddle through LDS after a plain load
        rp_rot_all<G, PP, NX, NT>(x, X, [&](int s) -> u32 { return rp_uniform(EXPT[s]); }, N, t);
    }

    // ---- levels ----------------------------------------------------------------------
#pragma unroll
    for (int li = 0; li < LOGG; ++li) {
        const int JB = DIR == 0 ? LOGG - 1 - li : li;
        // E == 0 for every pair of the level: the first DIF level of a pass (no pending
        // exponents yet, rp_pend(.., 0, ..) == 0, unless an earlier pass left its own) and the
        // first DIT level of the pass that holds the transform's last level (h == 1: rp_tw == 0).
        // Partners are then this thread's own registers -- no LDS round (workgroup-uniform).
        if ((DIR == 0 && li == 0) || (DIR == 1 && li == 0 && HL)) {
#pragma unroll
            for (int pi = 0; pi < G / 2; ++pi) {
                const int i = ((pi >> JB) << (JB + 1)) | (pi & ((1 << JB) - 1));
                const int k = i | (1 << JB);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const Pr y = x[k][r];
                    pr_bfly(x[i][r], x[k][r], x[i][r], y, false);
                }
            }
            if (li < 3) RP_STAMP(2 + li);
            continue;
        }
        // partner x_k read rotated by E: (x_i, x_k) <- (x_i + 2^E x_k, x_i - 2^E x_k)
        // Split pass: the input slots at or past zero_from are zero (zero_in is monotone in the
        // slot), so before DIF level li >= 1 slot s is zero iff input slot s mod 2^(LOGG - li)
        // was.  A zero partner is neither published nor read: (x_i, x_k) <- (x_i, x_i), bit for
        // bit what the butterfly gives (workgroup-uniform; C3's pass-0 groups hold 4-5 live
        // slots of 16, so level 1 exchanges 0-2 of its 8 pairs)
        auto pz = [&](int k) -> bool { return RP_SPLIT_ZSKIP && SPLIT && zero_in(k & ((1 << (LOGG - li)) - 1)); };
        const int tl = rp_launder(t);
        bool xch = false;
#pragma unroll
        for (int pi = 0; pi < G / 2; ++pi) {
            const int i = ((pi >> JB) << (JB + 1)) | (pi & ((1 << JB) - 1));
            if (pz(i | (1 << JB))) continue;
            rp_pub<PP, NT>(X, pi, x[i | (1 << JB)], tl);
            xch = true;
        }
        if (xch) __syncthreads();
#pragma unroll
        for (int pi = 0; pi < G / 2; ++pi) {
            const int i = ((pi >> JB) << (JB + 1)) | (pi & ((1 << JB) - 1));
            const int k = i | (1 << JB);
            if (pz(k)) {
#pragma unroll
                for (int r = 0; r < R; ++r) x[k][r] = x[i][r];
                continue;
            }
            const u32 E = rp_uniform(EXPT[2 * G + (G / 2) * li + pi]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r % 2 == 0) RP_FENCE();   // two partner reads in flight at a time
                bool ng;
                const Pr y = rp_get_al<PP>(X, pi, tl + NT * r, E, N, ng);
                pr_bfly(x[i][r], x[k][r], x[i][r], y, ng);
            }
        }
        if (xch) __syncthreads();
        if (li < 3) RP_STAMP(2 + li);
    }
    // the pending exponents of the last level (whole pairs): one aligned rotation round -- none
    // after the transform's last level (rp_pend_pos with hi == lbM is 0 for every position)
    if (DIR == 0 && !a.pkeep && a.lvl0 + LOGG < a.lbM) {
        rp_rot_all_al<G, PP, NX, NT>(x, X, [&](int s) -> u32 { return rp_uniform(EXPT[G + s]); }, N, t);
    }
    if (DIR == 1) rp_pin<G, R>(x);
    if (DIR == 1 && GX) {   // inverse MFA twiddle and/or fused scaling (bp_post)
        rp_rot_all<G, PP, NX, NT>(x, X, [&](int s) -> u32 { return rp_uniform(EXPT[s]); }, N, t);
    }
    RP_STAMP(5);

    // ---- store (reduced form) --------------------------------------------------------
    if (DIR == 1) rp_pin<G, R>(x);
    rp_store<G, G, PP, NT>(x, st, SLT, [&](int i) -> bool {
        const int bs = (g.pos0 + i * g.pstep) & ~(g.pstep - 1);
        return DIR == 1 || (bs < a.need && bs + g.pstep > a.need_lo);
    }, (short *)smem, t);
    if (FILL) {   // IFFT_radix2_truncate's fill (mul_fft.c:1760-1764): b_(p+h) = 2^(p rho) a_p for p >= t - h
        auto fills = [&](int s) -> bool { return g.pos0 + s * g.pstep >= a.fill_lo; };
        __syncthreads();   // every HX read of the store done (the rotation reuses the exchange slots)
        if (t < G) SLT[t] += (u32)((long)a.fill_off * a.pos_stride);
        rp_rot_all_al<G, PP, NX, NT>(x, X, [&](int s) -> u32 {
            return fills(s) ? (u32)(((u64)(g.pos0 + s * g.pstep) * a.fill_rho) % N2) : 0u;
        }, N, t);
        rp_store<G, G, PP, NT>(x, st, SLT, fills, (short *)smem, t);
    }
    RP_STAMP(6);
    if (stamp) {
        __syncthreads();
        RP_STAMP(7);
    }
#undef RP_STAMP
}

// ---- element-wise steps of the truncated inverse column transform --------------------
// k_rpair<PP, OP>: the k_pairop operations (IFFT_radix2_truncate(1)_twiddle's pair steps,
// mul_fft.c:1604-1668, :1733-1790) on the pair (i, i + h) of one column, in the register
// pair form: sums and differences are carry chains, the multipliers 2^e are rotations
// through one LDS exchange slot (aligned when e is a whole number of limb pairs, else the
// general 32-bit digit rotation; halving is 2^(2N-1)).  512 threads, 9 l bytes of LDS:
// several workgroups per CU overlap their loads and stores.
template <int PP, int OP>
__global__ __launch_bounds__(RP_NT) void k_rpair(PairArgs a)
{
    constexpr int l = 1024 * PP;
    constexpr bool LOADB = OP != OP_DOUBLE && OP != OP_FILL;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RX<PP> X{smem};
    u32 *SL = (u32 *)(smem + RX<PP>::SB);
    const int t = threadIdx.x;
    const int col = (int)(blockIdx.x % a.ncol);
    const int i = a.i0 + (int)(blockIdx.x / a.ncol);
    const u32 N = (u32)a.N, N2 = 2 * (u32)a.N;
    const u32 e = (u32)(((u64)i * a.rho) % N2);
    if (t < 2) SL[t] = (u32)((long)(a.off + i + (t ? a.h : 0)) * a.NC + col);
    __syncthreads();
    Coef st;
    st.dig = a.dig;
    st.cb = a.cb;
    st.top = a.top;
    unsigned short *CODE = (unsigned short *)smem;
    Pr x[2][PP];
    const RpCodes cd = rp_codes_load<LOADB ? 2 : 1, PP>(st, SL, t);
    rp_load_limbs<LOADB ? 2 : 1, 2, PP>(x, st, SL, t);
    rp_codes_store<LOADB ? 2 : 1, PP>(CODE, cd, t);
    __syncthreads();
    rp_decode<LOADB ? 2 : 1, 2, PP>(x, CODE, t);
    // y <- 2^E y through exchange slot 0 (E workgroup-uniform); barriers on both sides
    auto rot = [&](Pr(&y)[PP], u32 E) {
        if (E == 0) return;
        rp_pub<PP>(X, 0, y, t);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < PP; ++r) {
            RP_FENCE();
            if (E % 128 == 0) {
                bool ng;
                const Pr v = rp_get_al<PP>(X, 0, t + RP_NT * r, E, N, ng);
                y[r] = pr_cneg(v, ng);
            } else {
                y[r] = rp_get_rot<PP>(X, 0, t + RP_NT * r, E, N);
            }
        }
        __syncthreads();
    };
    switch (OP) {
    case OP_DOUBLE:   // a = 2a
#pragma unroll
        for (int r = 0; r < PP; ++r) x[0][r] = pr_add(x[0][r], x[0][r]);
        break;
    case OP_HALFADD:  // a = (a + b) / 2
#pragma unroll
        for (int r = 0; r < PP; ++r) x[0][r] = pr_add(x[0][r], x[1][r]);
        rot(x[0], N2 - 1);
        break;
    case OP_FILL:     // b = 2^e a
#pragma unroll
        for (int r = 0; r < PP; ++r) x[1][r] = x[0][r];
        rot(x[1], e);
        break;
    case OP_FIX:      // d = a - b; a = a + d; b = 2^e d
#pragma unroll
        for (int r = 0; r < PP; ++r) {
            const Pr d = pr_sub(x[0][r], x[1][r]);
            x[0][r] = pr_add(x[0][r], d);
            x[1][r] = d;
        }
        rot(x[1], e);
        break;
    case OP_TWOXMY:   // a = 2a - b
#pragma unroll
        for (int r = 0; r < PP; ++r) x[0][r] = pr_sub(pr_add(x[0][r], x[0][r]), x[1][r]);
        break;
    default:          // OP_IBFLY: t = 2^-e b; a, b = a + t, a - t
        rot(x[1], e ? N2 - e : 0);
#pragma unroll
        for (int r = 0; r < PP; ++r) pr_bfly(x[0][r], x[1][r], x[0][r], x[1][r], false);
        break;
    }
    __syncthreads();   // HX (rp_store) overlays the exchange slot and the codes
    rp_store<2, 2, PP>(x, st, SL, [&](int k) -> bool {
        return k == 0 ? OP != OP_FILL : (OP == OP_FILL || OP == OP_FIX || OP == OP_IBFLY);
    }, (short *)smem, t);
}

// ---- the tail of the truncated inverse in one kernel -------------------------------------
// k_rchain<PP, NB>: the recursion of IFFT_radix2_truncate1 (mul_fft.c:1604-1668) ends with
// NB steps a = 2a - b on the same rows A_i = off + i (partners at off + hb[j] + i, innermost
// first), and the enclosing IFFT_radix2_truncate(1) (:1733-1790) then runs its inverse
// butterfly with A as the bottom rows: t = 2^-e_i A, X, A = X + t, X - t (X_i = xoff + i).
// One launch reads the NB + 2 coefficients of a column once and writes two (Exec::chain; the
// separate k_rpair steps read 2 NB + 2 and write NB + 2).
template <int PP, int NB>
__global__ __launch_bounds__(RP_NT) void k_rchain(PairArgs a)
{
    constexpr int NS = NB + 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RX<PP> X{smem};
    u32 *SL = (u32 *)(smem + RX<PP>::SB);
    const int t = threadIdx.x;
    const int col = (int)(blockIdx.x % a.ncol);
    const int i = a.i0 + (int)(blockIdx.x / a.ncol);
    const u32 N = (u32)a.N, N2 = 2 * (u32)a.N;
    const u32 e = (u32)(((u64)i * a.rho) % N2);
    if (t < NS) {
        const long row = t == 0 ? a.off + i : t <= NB ? a.off + a.hb[t - 1] + i : a.xoff + i;
        SL[t] = (u32)(row * a.NC + col);
    }
    __syncthreads();
    Coef st;
    st.dig = a.dig;
    st.cb = a.cb;
    st.top = a.top;
    unsigned short *CODE = (unsigned short *)smem;
    Pr x[NS][PP];
    const RpCodes cd = rp_codes_load<NS, PP>(st, SL, t);
    rp_load_limbs<NS, NS, PP>(x, st, SL, t);
    rp_codes_store<NS, PP>(CODE, cd, t);
    __syncthreads();
    rp_decode<NS, NS, PP>(x, CODE, t);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < PP; ++r) x[0][r] = pr_sub(pr_add(x[0][r], x[0][r]), x[1 + j][r]);
    const u32 E = e ? N2 - e : 0;   // workgroup-uniform
    if (E) {
        rp_pub<PP>(X, 0, x[0], t);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < PP; ++r) {
            RP_FENCE();
            if (E % 128 == 0) {
                bool ng;
                const Pr v = rp_get_al<PP>(X, 0, t + RP_NT * r, E, N, ng);
                x[0][r] = pr_cneg(v, ng);
            } else {
                x[0][r] = rp_get_rot<PP>(X, 0, t + RP_NT * r, E, N);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < PP; ++r) pr_bfly(x[NS - 1][r], x[0][r], x[NS - 1][r], x[0][r], false);
    __syncthreads();   // HX (rp_store) overlays the exchange slot and the codes
    rp_store<NS, NS, PP>(x, st, SL, [&](int k) -> bool { return k == 0 || k == NS - 1; }, (short *)smem, t);
}

// ---- canonicalisation of a slot-form coefficient by all the waves of a workgroup -----------
// Wave-level: f[64 u0 ...] += sv (sub: -= sv), the carry rippling upward until it dies
// (almost always in the first limb); returns 1 if it ran off limb l - 1 (the value left
// [0, 2^N) upward, resp. downward).  Same ballot look-ahead as bp_canon.
__device__ int rp_ripple(const BSlot &b, int l, int u0, bool sub, u64 sv, int lane)
{
    const int rows = l >> 6;
    u64 run = 0;
    for (int u = u0; u < rows; ++u) {
        const int m = 64 * u + lane;
        const bool first = u == u0 && lane == 0;
        const u64 f = b.f[m];
        bool g, p;
        if (first) {
            u64 t2;
            g = sub ? f < sv : add_ovf(f, sv, &t2);
            p = sub ? f == sv : (f + sv) == MPF_MAXL;
        } else {
            g = false;
            p = sub ? f == 0 : f == MPF_MAXL;
        }
        const u64 X = __ballot(g), Yp = X | __ballot(p);
        u64 s1, s2;
        const bool o1 = add_ovf(X, Yp, &s1);
        const bool o2 = add_ovf(s1, run, &s2);
        const u64 add = (first ? sv : 0) + (((s2 ^ X ^ Yp) >> lane) & 1);
        b.f[m] = sub ? f - add : f + add;
        run = (o1 | o2) ? 1 : 0;
        if (!run) return 0;   // wave-uniform
    }
    return 1;
}

// bp_canon (mpn_normmod_2expp1, mul_fft.c:272) spread over NWV waves: wave w sweeps rows
// [w R, (w + 1) R) of the slot form (limb f_m + carry c_m into it) with no inc/dec chain
// entering its first row, the carry of the limb below computed directly.  A chain that
// leaves a segment (its run-out; probability ~2^-64 per boundary) is added afterwards at the
// next segment's first limb by rp_ripple, in order, by wave 0, which then folds the carry
// limb (value == f - top) as bp_canon does.  Returns the carry limb (1 only for 2^N) in
// wave 0; scr: 2 NWV + 1 ints of LDS.
template <int NWV>
__device__ int rp_canon_par(const BSlot &b, int l, int wave, int lane, int *scr)
{
    const int rows = l >> 6, R = rows / NWV, u0 = wave * R;
    int prevk = 0;
    if (u0) {   // carry out of limb 64 u0 - 1 (f + c), read before any wave rewrites it
        const u64 f = b.f[64 * u0 - 1];
        const int c = b.c[64 * u0 - 1];
        const u64 nf = f + (u64)(i64)c;
        prevk = c >= 0 ? (int)(nf < f) : -(int)(nf > f);
    }
    __syncthreads();
    u64 run1 = 0, run2 = 0;
    int topk = 0;
    for (int u = u0; u < u0 + R; ++u) {
        const int m = 64 * u + lane;
        const u64 f = b.f[m];
        const int c = b.c[m];
        u64 nf = f + (u64)(i64)c;
        const int k = c >= 0 ? (int)(nf < f) : -(int)(nf > f);   // carry out of limb m, in {-1, 0, 1}
        const int r = wv_ror1(k);
        const int cm = lane ? r : prevk;                          // carry into limb m
        prevk = wv_readlane(k, 63);
        if (u == rows - 1) topk = prevk;                          // out of the top limb: the carry limb
        const bool inc = cm == 1, dec = cm == -1;
        {
            const u64 X = __ballot(inc && nf == MPF_MAXL);
            const u64 Yp = X | __ballot(inc ? nf == MPF_MAXL - 1 : nf == MPF_MAXL);
            u64 s1, s2;
            const bool o1 = add_ovf(X, Yp, &s1);
            const bool o2 = add_ovf(s1, run1, &s2);
            nf += (u64)inc + (((s2 ^ X ^ Yp) >> lane) & 1);
            run1 = (o1 | o2) ? 1 : 0;
        }
        {
            const u64 X = __ballot(dec && nf == 0);
            const u64 Yp = X | __ballot(dec ? nf == 1 : nf == 0);
            u64 s1, s2;
            const bool o1 = add_ovf(X, Yp, &s1);
            const bool o2 = add_ovf(s1, run2, &s2);
            nf -= (u64)dec + (((s2 ^ X ^ Yp) >> lane) & 1);
            run2 = (o1 | o2) ? 1 : 0;
        }
        b.f[m] = nf;
    }
    if (lane == 0) {
        scr[2 * wave] = (int)run1;
        scr[2 * wave + 1] = (int)run2;
        if (wave == NWV - 1) scr[2 * NWV] = topk;
    }
    __syncthreads();
    if (wave != 0) return 0;
    int top = scr[2 * NWV] + scr[2 * (NWV - 1)] - scr[2 * (NWV - 1) + 1];
    for (int w = 1; w < NWV; ++w) {   // run-outs of the lower segments (w - 1): almost never
        const int d = scr[2 * (w - 1)] - scr[2 * (w - 1) + 1];
        if (d > 0) top += rp_ripple(b, l, w * R, false, 1, lane);
        if (d < 0) top -= rp_ripple(b, l, w * R, true, 1, lane);
    }
    if (top == 0) return 0;
    // value == f - top, f in [0, 2^N), |top| <= 3: one ripple from limb 0, then the 2^N case
    const bool sub = top > 0;
    if (!rp_ripple(b, l, 0, sub, (u64)(sub ? top : -top), lane)) return 0;
    // the ripple left 2^N: sub: f = 2^N + y - top >= 2^N - 3, true value f + 1;
    // add: f = y + |top| - 2^N in {0, 1, 2}, true value f - 1
    const u64 f0 = wv_readlane64(b.f[lane], 0);
    const bool to_2N = sub ? (f0 == MPF_MAXL) : (f0 == 0);
    if (to_2N) {
        for (int u = 0; u < rows; ++u) b.f[64 * u + lane] = 0;
        return 1;
    }
    if (lane == 0) b.f[0] = sub ? f0 + 1 : f0 - 1;
    return 0;
}

// ---- scaling by 2^-(depth+1) and canonicalisation (mul_fft.c:3256-3260) ----------------
// k_rscale<PP>: one coefficient per workgroup (many per CU, so one's load overlaps
// another's arithmetic): load into the register pair form, multiply by 2^e with one general
// rotation through LDS, then resolve every carry: the limbs go back to LDS in the k_bpass
// slot form (limb + carry into it) and the rows are swept (the ballot carry-lookahead of
// mpn_normmod_2expp1 :272) by all eight waves, one segment each (rp_canon_par);
// the canonical residue in [0, 2^N] is stored with zero carry masks and its carry limb.
// Coefficients [lo, hi) of the launch take exponent e2 instead of e (one launch for all rows).
template <int PP, int NT = RP_NT>
__global__ __launch_bounds__(NT) void k_rscale(u64 *dig, u64 *cb, int *top, u32 N, u32 e, u32 e2, u32 lo, u32 hi)
{
    if (blockIdx.x >= lo && blockIdx.x < hi) e = e2;   // itft's deferred doubling: those rows by 2^-depth
    constexpr int l = 1024 * PP, HP = l / 2, cbw = 2 * l / 64, R = rp_r(PP, NT);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RX<PP> X{smem};
    u32 *SL = (u32 *)(smem + RX<PP>::SB);
    const int t = threadIdx.x;
    if (t == 0) SL[0] = blockIdx.x;
    __syncthreads();
    Coef st;
    st.dig = dig;
    st.cb = cb;
    st.top = top;
    unsigned short *CODE = (unsigned short *)smem;
    Pr x[1][R];
    const RpCodes cd = rp_codes_load<1, PP>(st, SL, t);
    rp_load_limbs<1, 1, PP, NT>(x, st, SL, t);
    rp_codes_store<1, PP>(CODE, cd, t);
    __syncthreads();
    rp_decode<1, 1, PP, NT>(x, CODE, t);
    rp_pub<PP, NT>(X, 0, x[0], t);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) x[0][r] = rp_get_rot<PP>(X, 0, t + NT * r, e, N);
    __syncthreads();
    // k_bpass slot form: f_m, c_m = carry into limb m (the overflow of pair m/2 - 1 for even
    // m, minus the last pair's for m = 0: 2^N == -1), zero for odd m
    const BSlot b = bp_slot(smem, 0, l);
    short *hx = (short *)(smem + bp_slot_bytes(l));   // after the slot: HP pair overflows
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int pp = t + NT * r;
        *(rp_v4u *)(b.f + 2 * pp) = pr_words(x[0][r]);
        hx[pp] = (short)x[0][r].h;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int pp = t + NT * r;
        const int hv = hx[pp ? pp - 1 : HP - 1];
        *(short *)(b.c + 2 * pp) = (short)((pp ? hv : -hv) & 0xff);   // c_2pp = hin (|hin| < 128), c_2pp+1 = 0
    }
    __syncthreads();
    {
        const int tv = rp_canon_par<NT / 64>(b, l, t >> 6, t & 63, (int *)(smem + bp_slot_bytes(l) + (size_t)l));
        if (t == 0) SL[1] = (u32)tv;
    }
    __syncthreads();
    const long sl = blockIdx.x;
    u64 *dst = dig + (size_t)sl * l;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int pp = t + NT * r;
        *(rp_v4u *)(dst + 2 * pp) = *(const rp_v4u *)(b.f + 2 * pp);
    }
    for (int w = t; w < cbw; w += NT) cb[(size_t)sl * cbw + w] = 0;
    if (t == 0) top[sl] = (int)SL[1];
}
