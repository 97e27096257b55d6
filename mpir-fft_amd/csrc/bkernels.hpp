// bkernels.hpp -- LDS-resident radix-2^LOGG passes for big coefficients
// (512 <= l <= 4096 limbs, l % 64 == 0: the 10^9..10^10-bit configs C2-C4).
//
// Same work and HBM format as k_pass (kernels.hpp): one workgroup owns a butterfly
// group of G = 2^LOGG coefficients of one column or row and runs LOGG radix-2 levels
// of FFT_radix2_twiddle / FFT_radix2 / IFFT_radix2(_twiddle) (mul_fft.c:1397, :786,
// :1444, :1964) on it, with the MFA twiddles (README:89), the fused split
// (FFT_split_bits, :115) and the fused 2^-(depth+1) scaling (:3256-3260).
//
// Why a separate kernel: at l = 2048 a coefficient is 16 KB, so k_pass can keep only
// G = 4 of them in carry-save registers and rotate them one at a time through LDS
// (2 levels per HBM round trip at l = 2048, 1 at l = 4096).  Here the G coefficients
// live in LDS in a packed form of 9 bytes per limb -- G = 8 at l = 2048, 4 at 4096,
// 16 at 1024 (~147 KB) -- and never leave it between levels.  16 waves per workgroup:
// each level, the G/2 butterfly pairs are split over them by rows of 64 limbs.
//
// LDS form of a residue x mod p = 2^N + 1 ("hv form"): limbs f_m (u64) and a signed
// byte c_m per limb,
//     x = sum_m (f_m + c_m) 2^(64 m)   (mod p),
// c_m = the high part that limb m-1 overflowed into limb m (c_0 takes limb l-1's
// overflow negated, since 2^N == -1, plus the HBM carry limb).  Carry-save digits
// of x are D_2m = lo32(f_m) + c_m, D_2m+1 = hi32(f_m), and a level turns digit pairs
// back into (f, c) limb by limb -- every lane works on its own limb, no carry chain,
// no neighbour exchange.  Carries are resolved once per pass when the group is
// written back: locally into the HBM "reduced" form (carry masks, coeff.hpp), or
// fully (canonical residue in [0, 2^N], mpn_normmod_2expp1 :272) by one wave per
// coefficient sweeping its rows with ballot carry-lookahead.
//
// Multiplications by 2^e are never executed as separate steps: a butterfly output
// that must be multiplied by 2^e is stored as is with a *pending* exponent, and the
// next level reads it through a rotated LDS read (digit index permutation, sign
// flip past 2^N, sub-digit shift); exponents of successive rotations add mod 2N.
// Pending exponents are wave-uniform closed forms of the slot index (no arrays).
// The last level applies every remaining exponent on its reads and stores unrotated.
#pragma once
#include "wkernels.hpp"

#include "bdispatch.hpp"           // BP_MAXLOGG, BP_RMAX (rows of 64 limbs per wave per level), BP_LDS_MAX

__host__ __device__ constexpr size_t bp_slot_bytes(int l) { return ((size_t)l * 9 + 15) / 16 * 16; }

struct BSlot {
    u64 *f;
    signed char *c;
};

__device__ __forceinline__ BSlot bp_slot(unsigned char *lds, int s, int l)
{
    BSlot b;
    b.f = (u64 *)(lds + (size_t)s * bp_slot_bytes(l));
    b.c = (signed char *)(b.f + l);
    return b;
}

__device__ __forceinline__ i64 bp_cneg(i64 v, bool n) { return n ? -v : v; }

// bit j of x -> bit 2j of the result (Morton spread)
__device__ __forceinline__ u64 bp_spread(u32 x)
{
    u64 v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// low / high part of D * 2^b split at 32 bits (D a signed digit, 0 <= b < 32): D 2^b = hi 2^32 + lo
__device__ __forceinline__ i64 bp_lo(i64 D, int b) { return (i64)(((u64)(u32)D << b) & MPF_M32); }
__device__ __forceinline__ i64 bp_hi(i64 D, int b)
{
    return (i64)(((u64)(u32)D << b) >> 32) + (i64)((u64)(D >> 32) << b);
}

// digits (d0, d1) = (2m, 2m+1) of 2^e x mod p, x in slot b; e in [0, 2N), wave-uniform
__device__ __forceinline__ void bp_ld(const BSlot &b, u64 e, u64 N, int l, int m, i64 &d0, i64 &d1)
{
    if (e == 0) {
        const u64 f = b.f[m];
        d0 = (i64)(u32)f + b.c[m];
        d1 = (i64)(f >> 32);
        return;
    }
    bool sg = false;
    if (e >= N) {
        sg = true;
        e -= N;
    }
    const int y = (int)(e >> 5), sb = (int)(e & 31), Y = y >> 1;
    int jh = m - Y;                    // source limb of the low digit (y even) / high digit (y odd)
    const bool wh = jh < 0;
    jh += wh ? l : 0;
    const u64 fh = b.f[jh];
    const i64 h0 = (i64)(u32)fh + b.c[jh], h1 = (i64)(fh >> 32);
    if (sb == 0 && !(y & 1)) {         // limb-aligned: signed limb permutation
        d0 = bp_cneg(h0, wh != sg);
        d1 = bp_cneg(h1, wh != sg);
        return;
    }
    int jl = m - Y - 1;
    const bool wl = jl < 0;
    jl += wl ? l : 0;
    const u64 fl = b.f[jl];
    const i64 l0 = (i64)(u32)fl + b.c[jl], l1 = (i64)(fl >> 32);
    if (!(y & 1)) {
        d0 = bp_cneg(bp_lo(h0, sb), wh) + bp_cneg(bp_hi(l1, sb), wl);
        d1 = bp_cneg(bp_lo(h1, sb) + bp_hi(h0, sb), wh);
    } else {
        d0 = bp_cneg(bp_lo(l1, sb) + bp_hi(l0, sb), wl);
        d1 = bp_cneg(bp_lo(h0, sb), wh) + bp_cneg(bp_hi(l1, sb), wl);
    }
    d0 = bp_cneg(d0, sg);
    d1 = bp_cneg(d1, sg);
}

// digit pair -> (limb, overflow into the next limb):  d0 + d1 2^32 = f + hv 2^64  (|d| < 2^40)
__device__ __forceinline__ void bp_red(i64 d0, i64 d1, u64 &f, int &hv)
{
    const u64 b = (u64)(u32)d1 << 32;
    const u64 s = (u64)d0 + b;
    const bool wr = s < b;
    const int c0 = d0 < 0 ? (wr ? 0 : -1) : (wr ? 1 : 0);
    f = s;
    hv = (int)(d1 >> 32) + c0;
}

// e mod 2N for e < 8N (no 64-bit division: every caller adds at most a few reduced terms)
// A rotation 2^e mod p split into wave-uniform parts (make_rot): sign, digit shift y, bit
// shift sb, whole-limb shift Y = y / 2.  "Aligned" = a signed limb permutation.
struct BExp {
    bool sg;
    int y, sb, Y;
    bool al;
};

__device__ __forceinline__ BExp bp_exp(u64 e, u64 N)
{
    BExp x;
    x.sg = e >= N;
    if (x.sg) e -= N;
    x.y = (int)(e >> 5);
    x.sb = (int)(e & 31);
    x.Y = x.y >> 1;
    x.al = x.sb == 0 && !(x.y & 1);
    return x;
}

// the LDS words bp_ld reads for limb m: limb m - Y (and m - Y - 1 unless aligned), mod l
template <bool AL>
struct BRaw {
    u64 fh, fl;
    int ch, cl;
};
template <>
struct BRaw<true> {   // aligned: one source limb
    u64 fh;
    int ch;
};

template <bool AL>
__device__ __forceinline__ void bp_raw(const BSlot &b, const BExp &x, int l, int m, BRaw<AL> &r)
{
    int jh = m - x.Y;
    jh += jh < 0 ? l : 0;
    r.fh = b.f[jh];
    r.ch = b.c[jh];
    if constexpr (!AL) {
        int jl = m - x.Y - 1;
        jl += jl < 0 ? l : 0;
        r.fl = b.f[jl];
        r.cl = b.c[jl];
    }
}

// digits (2m, 2m+1) of 2^e x from the raw words (same math as bp_ld)
template <bool AL>
__device__ __forceinline__ void bp_dig(const BRaw<AL> &r, const BExp &x, int m, i64 &d0, i64 &d1)
{
    const bool wh = m - x.Y < 0;
    const i64 h0 = (i64)(u32)r.fh + r.ch, h1 = (i64)(r.fh >> 32);
    if constexpr (AL) {
        d0 = bp_cneg(h0, wh != x.sg);
        d1 = bp_cneg(h1, wh != x.sg);
        return;
    } else {
    const bool wl = m - x.Y - 1 < 0;
    const i64 l0 = (i64)(u32)r.fl + r.cl, l1 = (i64)(r.fl >> 32);
    const int sb = x.sb;
    if (!(x.y & 1)) {
        d0 = bp_cneg(bp_lo(h0, sb), wh) + bp_cneg(bp_hi(l1, sb), wl);
        d1 = bp_cneg(bp_lo(h1, sb) + bp_hi(h0, sb), wh);
    } else {
        d0 = bp_cneg(bp_lo(l1, sb) + bp_hi(l0, sb), wl);
        d1 = bp_cneg(bp_lo(h0, sb), wh) + bp_cneg(bp_hi(l1, sb), wl);
    }
    d0 = bp_cneg(d0, x.sg);
    d1 = bp_cneg(d1, x.sg);
    }
}

// One level's butterflies on BP_RMAX rows of one pair (i, k): out_i = 2^ai x_i + 2^bi x_k,
// out_k = 2^ak x_i - 2^bk x_k (FULL; otherwise ai = ak = 0, bi = bk).  All LDS reads of a
// batch of rows are issued before any is consumed; AL: every exponent limb-aligned.
template <bool AL, bool FULL>
__device__ __forceinline__ void bp_rows(const BSlot &si, const BSlot &sk, const BExp &xai, const BExp &xbi,
                                        const BExp &xak, const BExp &xbk, u64 ai, u64 bi, u64 ak, u64 bk,
                                        u64 N, int l, int u0, int lane, u64 (&fs)[BP_RMAX], u64 (&fd)[BP_RMAX],
                                        int (&hs)[BP_RMAX], int (&hd)[BP_RMAX])
{
    if constexpr (!AL) {   // general rotations (MFA twiddles, scaling): row by row
#pragma unroll
        for (int r = 0; r < BP_RMAX; ++r) {
            __builtin_amdgcn_sched_barrier(0);   // one row at a time (register pressure)
            const int m = 64 * (u0 + r) + lane;
            i64 a0, a1, b0, b1;
            bp_ld(si, ai, N, l, m, a0, a1);
            bp_ld(sk, bi, N, l, m, b0, b1);
            bp_red(a0 + b0, a1 + b1, fs[r], hs[r]);
            if constexpr (FULL) {
                bp_ld(si, ak, N, l, m, a0, a1);
                bp_ld(sk, bk, N, l, m, b0, b1);
            } else {
                si.f[m] = fs[r];   // slot i is read unrotated, by this wave only: its limb can go now
            }
            bp_red(a0 - b0, a1 - b1, fd[r], hd[r]);
        }
        return;
    } else {
    constexpr int RB = FULL ? BP_RMAX / 2 : BP_RMAX;
#pragma unroll
    for (int h = 0; h < BP_RMAX; h += RB) {
        __builtin_amdgcn_sched_barrier(0);
        BRaw<AL> ra[RB], rb[RB], rak[FULL ? RB : 1], rbk[FULL ? RB : 1];
#pragma unroll
        for (int q = 0; q < RB; ++q) {
            const int m = 64 * (u0 + h + q) + lane;
            bp_raw<AL>(si, xai, l, m, ra[q]);
            bp_raw<AL>(sk, xbi, l, m, rb[q]);
            if constexpr (FULL) {
                bp_raw<AL>(si, xak, l, m, rak[q]);
                bp_raw<AL>(sk, xbk, l, m, rbk[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < RB; ++q) {
            const int m = 64 * (u0 + h + q) + lane;
            i64 a0, a1, b0, b1;
            bp_dig<AL>(ra[q], xai, m, a0, a1);
            bp_dig<AL>(rb[q], xbi, m, b0, b1);
            bp_red(a0 + b0, a1 + b1, fs[h + q], hs[h + q]);
            if constexpr (FULL) {
                bp_dig<AL>(rak[q], xak, m, a0, a1);
                bp_dig<AL>(rbk[q], xbk, m, b0, b1);
            } else {
                si.f[m] = fs[h + q];   // slot i is read unrotated, by this wave only: its limb can go now
            }
            bp_red(a0 - b0, a1 - b1, fd[h + q], hd[h + q]);
        }
    }
    }
}

__device__ __forceinline__ u64 bp_mod2n(u64 e, u64 N2)
{
    e = e >= 2 * N2 ? e - 2 * N2 : e;
    return e >= N2 ? e - N2 : e;
}

// per-launch constants of a pass (the k_pass group geometry)
struct BGeo {
    int pos0, pstep;
    u64 tw0, twst;
    long sbase;
};

// level twiddle of the pair whose lower element is k at level index li (k_pass :212-229)
template <int LOGG, int DIR>
__device__ __forceinline__ u64 bp_tw(const PassArgs &a, const BGeo &g, int li, int k)
{
    const int JB = DIR == 0 ? LOGG - 1 - li : li;
    const int level = DIR == 0 ? a.lvl0 + li : a.lvl0 + LOGG - 1 - li;
    const int h = 1 << (a.lbM - level - 1);
    const u64 unit = a.rho << level;
    return (u64)(g.pos0 & (h - 1)) * unit + (u64)(k & ((1 << JB) - 1)) * (u64)g.pstep * unit;
}

// DIF: exponent pending on slot s after `done` levels.  Level j pairs (x, x | 2^JB_j),
// JB_j = LOGG-1-j, and leaves P'(x | 2^JB_j) = P(x) + t_j(x | 2^JB_j), P'(x) = P(x); so
// P_done(s) = P_0(s without its top `done` bits) + sum over the levels j whose bit
// JB_j is set in s of t_j(s without the bits of the later levels j+1 .. done-1).
template <int LOGG>
__device__ __forceinline__ u64 bp_pend(const PassArgs &a, const BGeo &g, int done, int s, u64 N2)
{
    const int base = s & ~(((1 << done) - 1) << (LOGG - done));
    u64 e = a.tw_mode == 1 ? bp_mod2n(g.tw0 + (u64)base * g.twst, N2) : 0;
    for (int j = 0; j < done; ++j)
        if ((s >> (LOGG - 1 - j)) & 1) {
            const int x = s & ~(((1 << (done - 1 - j)) - 1) << (LOGG - done));
            e = bp_mod2n(e + bp_tw<LOGG, 0>(a, g, j, x), N2);
        }
    return e;
}

// DIT: final multiplier of slot s (inverse MFA twiddle, fused scaling)
__device__ __forceinline__ u64 bp_post(const PassArgs &a, const BGeo &g, int s, u64 N2)
{
    u64 e = 0;
    if (a.tw_mode == 2) {
        const u64 t = bp_mod2n(g.tw0 + (u64)s * g.twst, N2);
        e = t ? N2 - t : 0;
    }
    if (a.scale_e) e = bp_mod2n(e + a.scale_e, N2);
    return e;
}

// One wave resolves slot b completely: canonical residue in [0, 2^N] left in b.f,
// returns the carry limb (1 only for 2^N).  Rows are swept in order with running
// carries; same method as wv_canon (wave.hpp) / mpn_normmod_2expp1 (mul_fft.c:272).
__device__ int bp_canon(const BSlot &b, int l, int lane)
{
    const int rows = l >> 6;
    u64 run1 = 0, run2 = 0;
    int prevk = 0, topk = 0;
    for (int u = 0; u < rows; ++u) {
        const int m = 64 * u + lane;
        const u64 f = b.f[m];
        const int c = b.c[m];
        u64 nf = f + (u64)(i64)c;
        const int k = c >= 0 ? (int)(nf < f) : -(int)(nf > f);   // carry out of limb m, in {-1, 0, 1}
        const int r = wv_ror1(k);
        const int cm = lane ? r : (u ? prevk : 0);                // carry into limb m
        prevk = wv_readlane(k, 63);
        if (u == rows - 1) topk = prevk;                          // out of the top limb: stays in the carry limb
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
    const int top = topk + (int)run1 - (int)run2;
    if (top == 0) return 0;
    // value == f - top, f in [0, 2^N), |top| <= 3: one carry/borrow chain from limb 0
    const bool sub = top > 0;
    const u64 sv = (u64)(sub ? top : -top);
    u64 run = 0;
    for (int u = 0; u < rows; ++u) {
        const int m = 64 * u + lane;
        const u64 f = b.f[m];
        bool g, p;
        if (m == 0) {
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
        const u64 add = (m == 0 ? sv : 0) + (((s2 ^ X ^ Yp) >> lane) & 1);
        b.f[m] = sub ? f - add : f + add;
        run = (o1 | o2) ? 1 : 0;
        if (!run) return 0;   // wave-uniform: the chain died, nothing above changes
    }
    // the chain left 2^N: sub: f = 2^N + y - top >= 2^N - 3, true value f + 1;
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

// GEN: some rotation of this pass is not a whole number of limbs (MFA twiddles with
// w % 64 != 0, the fused scaling); otherwise every level takes the batched aligned path.
template <int LOGG, int DIR, bool GEN>
__global__ __launch_bounds__(64 * BP_WAVES) void k_bpass(PassArgs a)
{
    pass_clear_flags(a);
    constexpr int G = 1 << LOGG;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = wv_lane();
    const int wave = wv_id();
    const int nt = blockDim.x, nwv = nt >> 6;
    const int l = a.l, rows = l >> 6, lrows = __builtin_ctz(rows);   // host: rows a power of two
    const u64 N = a.N, N2 = 2 * a.N;
    const int op = blockIdx.y;
    Coef st;
    st.dig = a.dig[op];
    st.cb = a.cb[op];
    st.top = a.top[op];
    const int sub = (int)(blockIdx.x / a.ngroups);
    const int grp = (int)(a.grp0 + blockIdx.x % a.ngroups);
    const int lobits = a.lbM - a.lvl0 - LOGG;
    const int lo = grp & ((1 << lobits) - 1);
    const int hi = grp >> lobits;
    const int bstart = hi << (a.lbM - a.lvl0);
    if (DIR == 0 && (bstart >= a.need || bstart + (1 << (a.lbM - a.lvl0)) <= a.need_lo)) return;   // whole block past the truncation point / outside the rows needed (workgroup-uniform)
    BGeo g;
    g.pos0 = bstart | lo;
    g.pstep = 1 << lobits;
    g.sbase = (long)sub * a.sub_stride;
    const u64 rsub = a.tw_mode ? (u64)revbin_dev(a.sub_off + sub, a.tw_lbR) : 0;
    g.tw0 = a.tw_w * (u64)(a.pos_off + g.pos0) * rsub;
    g.twst = a.tw_w * (u64)g.pstep * rsub;
    auto slot_of = [&](int i) -> long {
        const int ps = a.pos_off + g.pos0 + i * g.pstep;
        return g.sbase + (long)(ps >> a.pbb) * a.pbs + (long)(ps & ((1 << a.pbb) - 1)) * a.pos_stride;
    };
    int *ctop = (int *)(smem + (size_t)G * bp_slot_bytes(l));
    // diagnostics (MPFFT_BP_STAMPS): thread 0 stamps the phase boundaries of this workgroup
    unsigned long long *stamp = a.dbg ? a.dbg + 8 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) : nullptr;
    if (stamp && threadIdx.x == 0) stamp[0] = __builtin_amdgcn_s_memtime();

    // ---- load the group into LDS ------------------------------------------------------
    // 2-limb (16-byte) chunks; chunk c = tid + k nt is limbs 2p, 2p+1 of slot c / (l/2).
    // Each thread issues the loads of a batch of BP_LB chunks before it consumes any.
    {
        typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
        const int cps = l >> 1;                    // chunks per slot (power of two)
        const int lcps = __builtin_ctz(cps);
        const int K = (G * cps + nt - 1) / nt;     // chunks per thread (<= 2 BP_LB)
        for (int k0 = 0; k0 < K; k0 += BP_LB) {
            v2u v[BP_LB];
            u64 x2[BP_LB];
            v2u cw[BP_LB];
            int cprev[BP_LB];
#pragma unroll
            for (int kk = 0; kk < BP_LB; ++kk) {
                v[kk] = v2u{0, 0};
                x2[kk] = 0;
                cw[kk] = v2u{0, 0};
                cprev[kk] = 0;
                const int c = threadIdx.x + (k0 + kk) * nt;
                if (k0 + kk >= K || c >= G * cps) continue;
                const int i = c >> lcps, pp = c & (cps - 1);
                if (DIR == 0 && g.pos0 + i * g.pstep >= a.zero_from) continue;   // zero input
                if (a.src[op]) {   // first forward column pass: split fused into the load
                    const long j = (long)(a.pos_off + g.pos0 + i * g.pstep) * a.jNC + a.sub_off + sub;
                    const u64 off = (u64)j * a.bits1 + (u64)pp * 128;
                    const long q = (long)(off >> 6);
                    const long ns = a.nsrc[op];
                    const u64 *sp = a.src[op];
                    if ((u64)pp * 128 < a.bits1) {
                        const SrcSlice sv{a.src_chunk, a.jNC, a.sub_off};
                        v[kk].x = src_limb(sp, ns, sv, j, a.bits1, q);
                        v[kk].y = src_limb(sp, ns, sv, j, a.bits1, q + 1);
                        x2[kk] = src_limb(sp, ns, sv, j, a.bits1, q + 2);
                    }
                } else {
                    const long sl = slot_of(i);
                    v[kk] = *(const v2u *)(st.dig + (size_t)sl * l + 2 * pp);
                    const u64 *cbp = st.cb + (size_t)sl * cb_words(l);
                    const int W = (2 * pp) >> 6;
                    cw[kk] = *(const v2u *)(cbp + 2 * W);
                    if (!((2 * pp) & 63)) {   // carry into the row's first limb: bit 63 of the previous row
                        const int Wp = W ? W - 1 : rows - 1;
                        const v2u pv = *(const v2u *)(cbp + 2 * Wp);
                        cprev[kk] = (int)(pv.x >> 63) - (int)(pv.y >> 63);
                        if (!W) cprev[kk] = -cprev[kk] - st.top[sl];   // limb l-1's carry weighs 2^N == -1; + carry limb
                    }
                }
            }
#pragma unroll
            for (int kk = 0; kk < BP_LB; ++kk) {
                const int c = threadIdx.x + (k0 + kk) * nt;
                if (k0 + kk >= K || c >= G * cps) continue;
                const int i = c >> lcps, pp = c & (cps - 1);
                const BSlot b = bp_slot(smem, i, l);
                const int m = 2 * pp, bt = m & 63;
                int c0 = 0, c1 = 0;
                u64 f0 = v[kk].x, f1 = v[kk].y;
                if (a.src[op]) {
                    const u64 off = (u64)(a.pos_off + g.pos0 + i * g.pstep) * a.jNC * a.bits1 +
                                    (u64)(a.sub_off + sub) * a.bits1 + (u64)pp * 128;
                    const int sh = (int)(off & 63);
                    if (sh) {
                        f0 = (f0 >> sh) | (f1 << (64 - sh));
                        f1 = (f1 >> sh) | (x2[kk] << (64 - sh));
                    }
                    const u64 left = (u64)m * 64 < a.bits1 ? a.bits1 - (u64)m * 64 : 0;   // bits of this coefficient left
                    if (left < 64) f0 &= (((u64)1) << left) - 1;
                    if (left < 128) f1 = left <= 64 ? 0 : f1 & ((((u64)1) << (left - 64)) - 1);
                } else {
                    c0 = bt ? (int)((cw[kk].x >> (bt - 1)) & 1) - (int)((cw[kk].y >> (bt - 1)) & 1) : cprev[kk];
                    c1 = (int)((cw[kk].x >> bt) & 1) - (int)((cw[kk].y >> bt) & 1);
                }
                *(v2u *)(b.f + m) = v2u{f0, f1};
                *(short *)(b.c + m) = (short)((c0 & 0xff) | ((c1 & 0xff) << 8));
            }
        }
    }
    __syncthreads();
    if (stamp && threadIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memtime();

    // ---- levels -------------------------------------------------------------------
    const int wpp = rows / BP_RMAX;            // waves per butterfly pair; host launches (G/2) wpp waves
    const int pi = wave / wpp, u0 = (wave % wpp) * BP_RMAX;
    for (int li = 0; li < LOGG; ++li) {
        const int JB = DIR == 0 ? LOGG - 1 - li : li;
        const int i = ((pi >> JB) << (JB + 1)) | (pi & ((1 << JB) - 1));
        const int k = i | (1 << JB);
        const bool full = li == LOGG - 1;
        // out_i = 2^ai x_i + 2^bi x_k,  out_k = 2^ak x_i - 2^bk x_k
        u64 ai = 0, bi, ak = 0, bk;
        if (DIR == 0) {
            const u64 Pi = bp_pend<LOGG>(a, g, li, i, N2), Pk = bp_pend<LOGG>(a, g, li, k, N2);
            if (full) {
                const u64 t = bp_tw<LOGG, 0>(a, g, li, k);
                ai = Pi;
                bi = Pk;
                ak = bp_mod2n(Pi + t, N2);
                bk = bp_mod2n(Pk + t, N2);
            } else {
                bi = bk = Pk >= Pi ? Pk - Pi : Pk + N2 - Pi;
            }
        } else {
            const u64 t = bp_mod2n(bp_tw<LOGG, 1>(a, g, li, k), N2);
            const u64 E = t ? N2 - t : 0;
            if (full) {
                const u64 Fi = bp_post(a, g, i, N2), Fk = bp_post(a, g, k, N2);
                ai = Fi;
                bi = bp_mod2n(Fi + E, N2);
                ak = Fk;
                bk = bp_mod2n(Fk + E, N2);
            } else {
                bi = bk = E;
            }
        }
        const BSlot si = bp_slot(smem, i, l), sk = bp_slot(smem, k, l);
        const BExp xai = bp_exp(ai, N), xbi = bp_exp(bi, N), xak = bp_exp(ak, N), xbk = bp_exp(bk, N);
        u64 fs[BP_RMAX], fd[BP_RMAX];
        int hs[BP_RMAX], hd[BP_RMAX];
        if (!GEN) {
            if (!full) bp_rows<true, false>(si, sk, xai, xbi, xak, xbk, ai, bi, ak, bk, N, l, u0, lane, fs, fd, hs, hd);
            else bp_rows<true, true>(si, sk, xai, xbi, xak, xbk, ai, bi, ak, bk, N, l, u0, lane, fs, fd, hs, hd);
        } else if (!full) {
            bp_rows<false, false>(si, sk, xai, xbi, xak, xbk, ai, bi, ak, bk, N, l, u0, lane, fs, fd, hs, hd);
        } else {
            bp_rows<false, true>(si, sk, xai, xbi, xak, xbk, ai, bi, ak, bk, N, l, u0, lane, fs, fd, hs, hd);
        }
        __syncthreads();   // every read of this level is done before any slot is overwritten
#pragma unroll
        for (int r = 0; r < BP_RMAX; ++r) {
            const int m = 64 * (u0 + r) + lane;
            const int mn = m + 1 == l ? 0 : m + 1;
            if (full) si.f[m] = fs[r];
            sk.f[m] = fd[r];
            si.c[mn] = (signed char)(m + 1 == l ? -hs[r] : hs[r]);
            sk.c[mn] = (signed char)(m + 1 == l ? -hd[r] : hd[r]);
        }
        __syncthreads();
        if (stamp && threadIdx.x == 0 && li < 4) stamp[2 + li] = __builtin_amdgcn_s_memtime();
    }

    // ---- store --------------------------------------------------------------------
    if (a.canon) {
        for (int i = wave; i < G; i += nwv) {
            const int tv = bp_canon(bp_slot(smem, i, l), l, lane);
            if (lane == 0) ctop[i] = tv;
        }
        __syncthreads();
    }
    if (stamp && threadIdx.x == 0) stamp[6] = __builtin_amdgcn_s_memtime();
    // 128-limb blocks, 2 limbs per lane: 16-byte stores (one 1 KB wave instruction per block)
    const int cbw = cb_words(l);
    const int bpr = rows >> 1;                    // blocks per slot
    const int items = G * bpr;                    // wave t handles t, t + nwv, ...; batches of BP_SB
    typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
    for (int t0 = wave; t0 < items; t0 += BP_SB * nwv) {
        v2u f[BP_SB];
        short c[BP_SB];
#pragma unroll
        for (int q = 0; q < BP_SB; ++q) {
            const int t = t0 + q * nwv;
            f[q] = v2u{0, 0};
            c[q] = 0;
            if (t < items) {
                const int i = t >> (lrows - 1), v = t & (bpr - 1);
                const BSlot b = bp_slot(smem, i, l);
                const int m = 128 * v + 2 * lane;
                f[q] = *(const v2u *)(b.f + m);
                c[q] = a.canon ? 0 : *(const short *)(b.c + m);
            }
        }
#pragma unroll
        for (int q = 0; q < BP_SB; ++q) {
            const int t = t0 + q * nwv;
            if (t >= items) continue;
            const int i = t >> (lrows - 1), v = t & (bpr - 1);
            const int bs = (g.pos0 + i * g.pstep) & ~(g.pstep - 1);
            const bool keep = DIR == 1 || (bs < a.need && bs + g.pstep > a.need_lo);
            if (!keep) continue;   // wave-uniform
            const long sl = wv_uniform(slot_of(i));
            const int m = 128 * v + 2 * lane;
            u64 *dst = st.dig + (size_t)sl * l;
            u64 *cbp = st.cb + (size_t)sl * cbw;
            // f_m + c_m = nf + kout 2^64: limb + carry out of limb m (mask bit m; out of
            // limb l-1 it weighs 2^N == -1, as load_coeff reads it back).  Canonical: c == 0.
            const int c0 = (signed char)(c[q] & 0xff), c1 = (signed char)((unsigned short)c[q] >> 8);
            const u64 n0 = f[q].x + (u64)(i64)c0, n1 = f[q].y + (u64)(i64)c1;
            const int k0 = c0 >= 0 ? (int)(n0 < f[q].x) : -(int)(n0 > f[q].x);
            const int k1 = c1 >= 0 ? (int)(n1 < f[q].y) : -(int)(n1 > f[q].y);
            *(v2u *)(dst + m) = v2u{n0, n1};
            // mask words of rows 2v (lanes 0..31) and 2v+1: even/odd limb ballots, bit-interleaved
            const u64 pe = __ballot(k0 == 1), po = __ballot(k1 == 1);
            const u64 ne = __ballot(k0 == -1), no = __ballot(k1 == -1);
            if (lane < 2) {
                const int sh = 32 * lane;
                const u64 pw = bp_spread((u32)(pe >> sh)) | (bp_spread((u32)(po >> sh)) << 1);
                const u64 nw = bp_spread((u32)(ne >> sh)) | (bp_spread((u32)(no >> sh)) << 1);
                *(v2u *)(cbp + 4 * v + 2 * lane) = v2u{pw, nw};
            }
            if (v == 0 && lane == 0) st.top[sl] = a.canon ? ctop[i] : 0;
        }
    }
    if (stamp) {
        __syncthreads();
        if (threadIdx.x == 0) stamp[7] = __builtin_amdgcn_s_memtime();
    }
}
