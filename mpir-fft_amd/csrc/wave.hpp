// wave.hpp -- wave-owned coefficients (gfx950, wave64): one wavefront holds whole
// residues mod p = 2^N + 1 of l limbs, 64 (U-1) < l <= 64 U, so a pass never needs a
// workgroup barrier.
//
// Ownership: lane t of the wave holds limbs m = 64 u + t (u < U), i.e. carry-save
// digits 2m, 2m+1 (coeff.hpp "in-kernel" representation) in x[2u], x[2u+1].  A
// 64-limb row is one coalesced 512-byte global access per u.  The last limb l-1 is
// in row U-1.  F ("full") = compile-time l == 64 U: no per-lane limb masks at all.
//
// What the workgroup kernels (coeff.hpp) do with LDS scans and __syncthreads,
// these do inside the wave:
//   neighbour limb      DPP wave_ror:1 (lane t <- lane t-1, lane 0 <- lane 63 of
//                       the previous 64-limb row)
//   carry lookahead     64-bit ballots + one scalar add per row (generate = g,
//                       propagate = p: the carries of G + (G|P) + cin)
//   rotations (2^e)     per-wave LDS staging; LDS ops of one wave execute in order,
//                       so a compiler fence between write and read is enough
#pragma once
#include "coeff.hpp"

// lane t <- lane t-1, lane 0 <- lane 63
__device__ __forceinline__ int wv_ror1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x13C, 0xF, 0xF, false); }

__device__ __forceinline__ int wv_readlane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

__device__ __forceinline__ u64 wv_readlane64(u64 v, int lane)
{
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, lane);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), lane);
    return ((u64)hi << 32) | lo;
}

// a value the whole wave agrees on, as a scalar (lets the compiler use s_load for it)
__device__ __forceinline__ long wv_uniform(long v)
{
    const u32 lo = (u32)__builtin_amdgcn_readfirstlane((int)(u32)(u64)v);
    const u32 hi = (u32)__builtin_amdgcn_readfirstlane((int)(u32)((u64)v >> 32));
    return (long)(((u64)hi << 32) | lo);
}

// keeps the compiler from moving LDS accesses of other lanes across this point
__device__ __forceinline__ void wv_fence()
{
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// conditional negate without a 64-bit multiply
__device__ __forceinline__ i64 wv_cneg(i64 v, bool neg) { return neg ? -v : v; }

template <bool F>
__device__ __forceinline__ bool wv_in(int m, int l) { return F || m < l; }

// ---------------------------------------------------------------------------
// HBM <-> digits (same Coef format as coeff.hpp: limbs + carry masks + top;
// cb_words(l) == 2U here)
// ---------------------------------------------------------------------------
// Loads are split in two phases so that a wave issues the loads of all its
// coefficients before it waits for any: wv_load_raw issues the limb rows plus one
// vector load of the carry masks (lane u < U gets row u's two mask words) and the
// carry limb; wv_load_digits turns them into carry-save digits.
template <int U>
struct WvRaw {
    u64 v[U];
    u64 cbp, cbn;   // lane u < U: row u's +1 / -1 carry masks
    int top;
};

template <int U, bool F>
__device__ __forceinline__ void wv_load_raw(WvRaw<U> &r, const Coef &s, long slot, int l, int lane)
{
    slot = wv_uniform(slot);
    const u64 *p = s.dig + (size_t)slot * (size_t)l;
    const u64 *cbp = s.cb + (size_t)slot * (size_t)(2 * U);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        r.v[u] = wv_in<F>(m, l) ? p[m] : 0;
    }
    typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
    v2u c = {0, 0};
    if (lane < U) c = *(const v2u *)(cbp + 2 * lane);
    r.cbp = c.x;
    r.cbn = c.y;
    r.top = lane == 0 ? s.top[slot] : 0;
}

template <int U, bool F>
__device__ __forceinline__ void wv_load_digits(i64 (&d)[2 * U], const WvRaw<U> &r, int l, int lane)
{
    u64 pp = 0, pn = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        const u64 pw = wv_readlane64(r.cbp, u), nw = wv_readlane64(r.cbn, u);
        // carry into limb m = carry out of limb m - 1 (lane 0: bit 63 of the previous row)
        const i64 cin = lane ? (i64)((pw >> (lane - 1)) & 1) - (i64)((nw >> (lane - 1)) & 1)
                             : (i64)(pp >> 63) - (i64)(pn >> 63);
        pp = pw;
        pn = nw;
        d[2 * u] = wv_in<F>(m, l) ? (i64)(r.v[u] & MPF_M32) + cin : 0;
        d[2 * u + 1] = wv_in<F>(m, l) ? (i64)(r.v[u] >> 32) : 0;
    }
    // carry limb plus the carry out of limb l-1 (pp/pn = row U-1 now): both weigh 2^N == -1
    const int b = (l - 1) & 63;
    const i64 cl = (i64)((pp >> b) & 1) - (i64)((pn >> b) & 1) + r.top;
    if (lane == 0) d[0] -= cl;
}

template <int U, bool F>
__device__ __forceinline__ void wv_load(i64 (&d)[2 * U], const Coef &s, long slot, int l, int lane)
{
    WvRaw<U> r;
    wv_load_raw<U, F>(r, s, slot, l, lane);
    wv_load_digits<U, F>(d, r, l, lane);
}

// fused split (FFT_split_bits, mul_fft.c:115-170)
template <int U, bool F>
__device__ __forceinline__ void wv_load_split(i64 (&d)[2 * U], const u64 *src, long nsrc, const SrcSlice &sv, long j,
                                              u64 bits1, int l, int lane)
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        u64 v = 0;
        if (wv_in<F>(m, l) && (u64)m * 64 < bits1) {
            const u64 off = (u64)j * bits1 + (u64)m * 64;
            const long q = (long)(off >> 6);
            const int s = (int)(off & 63);
            const u64 w0 = src_limb(src, nsrc, sv, j, bits1, q);
            const u64 w1 = s ? src_limb(src, nsrc, sv, j, bits1, q + 1) : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
            const u64 left = bits1 - (u64)m * 64;
            if (left < 64) v &= (((u64)1) << left) - 1;
        }
        d[2 * u] = (i64)(v & MPF_M32);
        d[2 * u + 1] = (i64)(v >> 32);
    }
}

template <int U, bool F>
__device__ __forceinline__ void wv_store(const u64 (&f)[U], const int (&cc)[U], int topv, const Coef &s, long slot,
                                         int l, int lane)
{
    slot = wv_uniform(slot);
    u64 *p = s.dig + (size_t)slot * (size_t)l;
    u64 *cbp = s.cb + (size_t)slot * (size_t)(2 * U);
    // lane u < U stores row u's two carry masks (16 bytes): one store instruction
    int w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (wv_in<F>(m, l)) p[m] = f[u];
        const u64 pm = __ballot(wv_in<F>(m, l) && cc[u] == 1);
        const u64 nm = __ballot(wv_in<F>(m, l) && cc[u] == -1);
        if (lane == u) {
            w0 = (int)(u32)pm;
            w1 = (int)(u32)(pm >> 32);
            w2 = (int)(u32)nm;
            w3 = (int)(u32)(nm >> 32);
        }
    }
    typedef int v4i __attribute__((ext_vector_type(4)));
    if (lane < U) {
        v4i v;
        v.x = w0;
        v.y = w1;
        v.z = w2;
        v.w = w3;
        *(v4i *)(cbp + 2 * lane) = v;
    }
    if (lane == 0) s.top[slot] = topv;
}

// ---------------------------------------------------------------------------
// digits -> "reduced" limbs: f (u64) + carries cc in {-1,0,1} out of each limb,
// value = sum f_m 2^(64m) + sum cc_m 2^(64(m+1))  (|d| < 2^62)
// ---------------------------------------------------------------------------
template <int U, bool F>
__device__ __forceinline__ void wv_reduce(const i64 (&d)[2 * U], u64 (&f)[U], int (&cc)[U], int l, int lane)
{
    int hv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        // v = d0 + d1 2^32 = (d0 + lo32(d1) 2^32) + hi(d1) 2^64
        const i64 d0 = d[2 * u], d1 = d[2 * u + 1];
        const u64 b = (u64)(u32)d1 << 32;
        const u64 s = (u64)d0 + b;
        const bool wr = s < b;
        const i64 c0 = d0 < 0 ? (wr ? 0 : -1) : (wr ? 1 : 0);
        f[u] = wv_in<F>(m, l) ? s : 0;
        hv[u] = wv_in<F>(m, l) ? (int)((d1 >> 32) + c0) : 0;   // |hv| < 2^30
    }
    // the top limb's overflow wraps negated into limb 0
    const int hlast = wv_readlane(hv[U - 1], (l - 1) & 63);
    int rprev = -hlast;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        const int r = wv_ror1(hv[u]);
        const i64 pv = lane ? r : rprev;
        rprev = r;
        const u64 nf = f[u] + (u64)pv;
        const int c = pv >= 0 ? (int)(nf < f[u]) : -(int)(nf > f[u]);
        f[u] = wv_in<F>(m, l) ? nf : 0;
        cc[u] = wv_in<F>(m, l) ? c : 0;
    }
}

// binary carry lookahead over the U rows: carry into each lane's limb, returns carry out
template <int U>
__device__ __forceinline__ u32 wv_scan(const bool (&g)[U], const bool (&p)[U], u32 (&ci)[U], u32 cin, int lane)
{
    u64 run = cin;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u64 X = __ballot(g[u]);
        const u64 Y = X | __ballot(p[u]);
        u64 s1, s2;
        const bool o1 = add_ovf(X, Y, &s1);
        const bool o2 = add_ovf(s1, run, &s2);
        const u64 C = s2 ^ X ^ Y;
        ci[u] = (u32)((C >> lane) & 1);
        run = (o1 | o2) ? 1 : 0;
    }
    return (u32)run;
}

// reduced (f, cc) -> canonical residue in [0, 2^N] (mpn_normmod_2expp1, mul_fft.c:272-294);
// returns the carry limb (1 only for exactly 2^N, then f == 0)
template <int U, bool F>
__device__ __forceinline__ int wv_canon(u64 (&f)[U], const int (&cc)[U], int l, int lane)
{
    int top = wv_readlane(cc[U - 1], (l - 1) & 63);   // carry out of the top limb stays in the carry limb
    bool inc[U], dec[U], g[U], p[U];
    u32 ci[U];
    int rprev = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        const int r = wv_ror1(cc[u]);
        const int cm = lane ? r : rprev;
        rprev = r;
        inc[u] = wv_in<F>(m, l) && cm == 1;
        dec[u] = wv_in<F>(m, l) && cm == -1;
        g[u] = inc[u] && f[u] == MPF_MAXL;
        p[u] = wv_in<F>(m, l) ? (inc[u] ? f[u] == MPF_MAXL - 1 : f[u] == MPF_MAXL) : true;
    }
    top += (int)wv_scan<U>(g, p, ci, 0, lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (wv_in<F>(m, l)) f[u] += (u64)inc[u] + ci[u];
        g[u] = dec[u] && f[u] == 0;
        p[u] = wv_in<F>(m, l) ? (dec[u] ? f[u] == 1 : f[u] == 0) : true;
    }
    top -= (int)wv_scan<U>(g, p, ci, 0, lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (wv_in<F>(m, l)) f[u] -= (u64)dec[u] + ci[u];
    }
    if (top == 0) return 0;   // wave-uniform
    // value == f - top, f in [0, 2^N), |top| <= 2
    const bool sub = top > 0;
    const u64 sv = (u64)(sub ? top : -top);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (!wv_in<F>(m, l)) {
            g[u] = false;
            p[u] = true;
        } else if (m == 0) {
            u64 t2;
            g[u] = sub ? f[u] < sv : add_ovf(f[u], sv, &t2);
            p[u] = sub ? f[u] == sv : (f[u] + sv) == MPF_MAXL;
        } else {
            g[u] = false;
            p[u] = sub ? f[u] == 0 : f[u] == MPF_MAXL;
        }
    }
    const u32 co = wv_scan<U>(g, p, ci, 0, lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        const u64 add = (m == 0 ? sv : 0) + ci[u];
        if (wv_in<F>(m, l)) f[u] = sub ? f[u] - add : f[u] + add;
    }
    if (!co) return 0;
    // sub: f = 2^N + y - top >= 2^N - 2, true value f + 1.
    // add: f = y + |top| - 2^N in {0, 1}, true value f - 1.
    const u64 f0 = wv_readlane64(f[0], 0);
    const bool to_2N = sub ? (f0 == MPF_MAXL) : (f0 == 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (to_2N) f[u] = 0;
        else if (m == 0) f[u] = sub ? f[u] + 1 : f[u] - 1;
    }
    return to_2N ? 1 : 0;
}

template <int U, bool F>
__device__ __forceinline__ void wv_normalize_store(const i64 (&d)[2 * U], bool canon, const Coef &st, long slot,
                                                   int l, int lane)
{
    u64 f[U];
    int cc[U];
    wv_reduce<U, F>(d, f, cc, l, lane);
    int topv = 0;
    if (canon) {
        topv = wv_canon<U, F>(f, cc, l, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) cc[u] = 0;
    }
    wv_store<U, F>(f, cc, topv, st, slot, l, lane);
}

// ---------------------------------------------------------------------------
// rotations: x <- x * 2^e mod p through this wave's LDS staging buffer (2l i64)
// ---------------------------------------------------------------------------
template <int U, bool F>
__device__ __forceinline__ void wv_rot_write(const i64 (&x)[2 * U], i64 *stage, int l, int lane)
{
    typedef long long v2i __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (wv_in<F>(m, l)) {
            v2i v;
            v.x = x[2 * u];
            v.y = x[2 * u + 1];
            *(v2i *)(stage + 2 * m) = v;   // one ds_write_b128 per limb
        }
    }
}

template <int U, bool F>
__device__ __forceinline__ void wv_rot_read(i64 (&x)[2 * U], const i64 *stage, const Rot &r, int l, int lane)
{
    typedef long long v2i __attribute__((ext_vector_type(2)));
    const int L = 2 * l;
    const bool nsg = r.sgn < 0;
    if (r.b == 0 && !(r.y & 1)) {
        // limb-aligned (every FFT twiddle when w NC, w NR are multiples of 64): a signed
        // limb permutation, one 16-byte LDS read per limb
        const int yl = r.y >> 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = 64 * u + lane;
            if (wv_in<F>(m, l)) {
                int k = m - yl;
                const bool wrap = k < 0;
                k += wrap ? l : 0;
                const v2i v = *(const v2i *)(stage + 2 * k);
                const bool ng = wrap != nsg;
                x[2 * u] = wv_cneg(v.x, ng);
                x[2 * u + 1] = wv_cneg(v.y, ng);
            }
        }
        return;
    }
    if (r.b == 0) {   // digit-aligned: signed digit permutation
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = 64 * u + lane;
            if (wv_in<F>(m, l)) {
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    int k = 2 * m + v - r.y;
                    const bool wrap = k < 0;
                    k += wrap ? L : 0;
                    x[2 * u + v] = wv_cneg(stage[k], wrap != nsg);
                }
            }
        }
        return;
    }
    // general: 2^e = (-1)^sgn 2^(32 y + b); digit j takes lo(d_{j-y} << b) + hi(d_{j-y-1} << b),
    // each negated when its source wrapped past 2^N (rot_digit, coeff.hpp)
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = 64 * u + lane;
        if (wv_in<F>(m, l)) {
            int k = 2 * m - r.y;   // source of digit 2m's low part; km, kp its neighbours
            int km = k - 1, kp = k + 1;
            const bool wm = km < 0, w0 = k < 0, wp = kp < 0;
            km += wm ? L : 0;
            k += w0 ? L : 0;
            kp += wp ? L : 0;
            const i64 xm = stage[km], x0 = stage[k], xp = stage[kp];
            const u64 l0 = (u64)(u32)x0 << r.b, lm = (u64)(u32)xm << r.b, lp = (u64)(u32)xp << r.b;
            const i64 p0 = (i64)(l0 & MPF_M32), pp = (i64)(lp & MPF_M32);
            const i64 hm = (i64)(lm >> 32) + (i64)((u64)(xm >> 32) << r.b);
            const i64 h0 = (i64)(l0 >> 32) + (i64)((u64)(x0 >> 32) << r.b);
            x[2 * u] = wv_cneg(wv_cneg(p0, w0) + wv_cneg(hm, wm), nsg);
            x[2 * u + 1] = wv_cneg(wv_cneg(pp, wp) + wv_cneg(h0, w0), nsg);
        }
    }
}

// x[i] <- x[i] * 2^efn(i) for the i with sel(i) (compile-time after unrolling),
// staged in LDS slot slot(i) of this wave's buffer (2l i64 each)
template <int U, bool F, int G, typename SEL, typename SLOT, typename EF>
__device__ __forceinline__ void wv_rot_set(i64 (&x)[G][2 * U], SEL sel, SLOT slot, EF efn, u64 N, int l,
                                           i64 *stage, int lane)
{
    bool any = false;
#pragma unroll
    for (int i = 0; i < G; ++i) {
        if (!sel(i)) continue;
        if (efn(i)) {
            wv_rot_write<U, F>(x[i], stage + (size_t)slot(i) * 2 * l, l, lane);
            any = true;
        }
    }
    if (!any) return;
    wv_fence();
#pragma unroll
    for (int i = 0; i < G; ++i) {
        if (!sel(i)) continue;
        const u64 e = efn(i);
        if (e) wv_rot_read<U, F>(x[i], stage + (size_t)slot(i) * 2 * l, make_rot(e, N), l, lane);
    }
    wv_fence();
}

// every one of the G coefficients, in rounds of NS staging slots
template <int U, bool F, int G, int NS, int R0, typename EF>
__device__ __forceinline__ void wv_rot_all(i64 (&x)[G][2 * U], EF efn, u64 N, int l, i64 *stage, int lane)
{
    wv_rot_set<U, F, G>(x, [](int i) { return i >= R0 && i < R0 + NS; }, [](int i) { return i - R0; }, efn, N, l,
                        stage, lane);
    if constexpr (R0 + NS < G) wv_rot_all<U, F, G, NS, R0 + NS>(x, efn, N, l, stage, lane);
}

// the set sel (compact slot indices slot(i) < G/2) in rounds of NS staging slots
template <int U, bool F, int G, int NS, int R0, typename SEL, typename SLOT, typename EF>
__device__ __forceinline__ void wv_rot_rounds(i64 (&x)[G][2 * U], SEL sel, SLOT slot, EF efn, u64 N, int l,
                                              i64 *stage, int lane)
{
    constexpr int H = G > 1 ? G / 2 : 1;
    wv_rot_set<U, F, G>(x, [&](int i) { return sel(i) && slot(i) >= R0 && slot(i) < R0 + NS; },
                        [&](int i) { return slot(i) - R0; }, efn, N, l, stage, lane);
    if constexpr (R0 + NS < H) wv_rot_rounds<U, F, G, NS, R0 + NS>(x, sel, slot, efn, N, l, stage, lane);
}
