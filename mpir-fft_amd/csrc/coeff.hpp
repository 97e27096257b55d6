// coeff.hpp -- workgroup-level arithmetic on one residue modulo p = 2^N + 1 (gfx950, wave64).
//
// Representation (DESIGN.md "Data layout"):
//   HBM    : a coefficient is l 64-bit limbs (little endian) plus a signed "carry
//            limb" kept in a separate int32 array, value = limbs + top * 2^N.  This
//            is the reference's (l+1)-limb two's-complement block (README:54,
//            mul_fft.c:269-294) with the carry limb split out so every coefficient
//            body is a dense, 64-byte aligned l*8-byte run.
//   in-kernel: the N bits as L = 2l signed 32-bit *digits* held in int64
//            ("carry-save"), value = sum_j d_j 2^(32 j) mod p.  Additions and
//            subtractions are digit-wise with no carry chain; multiplication by
//            2^e mod p (the butterfly twiddle) is a digit permutation with
//            negated wrap plus a sub-digit shift split into lo/mid/hi parts
//            (rot_digit), so a whole multi-level pass runs without carries.
//            Carries are resolved once per pass by wg_normalize, a workgroup
//            carry-lookahead built on 64-lane ballots.
//
// Thread ownership: thread t owns limbs m = u * blockDim.x + t (u < U), i.e. digits
// 2m and 2m+1.  Consecutive lanes own consecutive limbs, so HBM traffic is
// 8 B/lane coalesced.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;
typedef __int128 i128;
typedef unsigned __int128 u128;

#define MPF_M32 0xFFFFFFFFull
#define MPF_MAXL 0xFFFFFFFFFFFFFFFFull

struct WG {
    int t, nt, lane, wave, nw;
};

__device__ __forceinline__ WG wg_ctx()
{
    WG c;
    c.t = threadIdx.x;
    c.nt = blockDim.x;
    c.lane = c.t & 63;
    c.wave = c.t >> 6;
    c.nw = c.nt >> 6;
    return c;
}

__device__ __forceinline__ bool add_ovf(u64 a, u64 b, u64 *s) { return __builtin_add_overflow(a, b, s); }

// ---------------------------------------------------------------------------
// Workgroup carry-lookahead over the l limbs of one coefficient.
//   g (bit u): limb u*nt+t generates a carry; p (bit u): it propagates one.
//   cin: carry into limb 0.  Returns bit u = carry into limb u*nt+t;
//   *cout = carry out of the last limb.  Limbs that do not exist must have
//   g = 0, p = 1.  Lane level: a 64-bit add of the ballot masks (generate = 2,
//   propagate = 1) gives every lane's carry in one instruction; entry level
//   (one entry per (u, wave)) the same trick in wave 0.
// scr: >= 3 * U * nw + 1 u64 of LDS.
// ---------------------------------------------------------------------------
template <int U>
__device__ u32 wg_scan(const WG &c, u32 g, u32 p, u32 cin, u32 *cout, u64 *scr)
{
    const int E = U * c.nw;
    u64 Gm[U], Pm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        Gm[u] = __ballot((g >> u) & 1);
        Pm[u] = __ballot((p >> u) & 1);
        if (c.lane == 0) {
            scr[2 * (u * c.nw + c.wave)] = Gm[u];
            scr[2 * (u * c.nw + c.wave) + 1] = Pm[u];
        }
    }
    __syncthreads();
    if (c.wave == 0) {
        u64 run = cin;
        for (int base = 0; base < E; base += 64) {
            int e = base + c.lane;
            bool eg = false, ep = true;
            if (e < E) {
                u64 X = scr[2 * e], Y = X | scr[2 * e + 1], s, s2;
                bool o0 = add_ovf(X, Y, &s);
                bool o1 = o0 | add_ovf(s, 1, &s2);
                eg = o0;
                ep = o1 && !o0;
            }
            u64 X = __ballot(eg), Y = X | __ballot(ep), s, s2;
            bool o = add_ovf(X, Y, &s);
            o |= add_ovf(s, run, &s2);
            u64 CI = s2 ^ X ^ Y;
            if (e < E) scr[2 * E + e] = (CI >> c.lane) & 1;
            run = o ? 1 : 0;
        }
        if (c.lane == 0) scr[3 * E] = run;
    }
    __syncthreads();
    u32 res = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u64 ci = scr[2 * E + u * c.nw + c.wave];
        u64 X = Gm[u], Y = Gm[u] | Pm[u], s, s2;
        add_ovf(X, Y, &s);
        add_ovf(s, ci, &s2);
        u64 C = s2 ^ X ^ Y;
        res |= (u32)((C >> c.lane) & 1) << u;
    }
    *cout = (u32)scr[3 * E];
    __syncthreads();
    return res;
}

// ---------------------------------------------------------------------------
// Resolve carry-save digits into limbs.
//   d[2u], d[2u+1]: digits 2m, 2m+1 of limb m = u*nt+t (|d| < 2^62).
//   Out: y[u] limbs, return value top, with value = y + top * 2^N (mod p).
//   canon = false: top in [-2, 2] ("reduced", what the next pass reloads).
//   canon = true : canonical residue in [0, 2^N] (top in {0,1}, top == 1 only
//                  for exactly 2^N), i.e. mpn_normmod_2expp1 (mul_fft.c:272).
// sh: >= l i64 of LDS; scr: scan scratch.  Contains barriers: call uniformly.
// ---------------------------------------------------------------------------
template <int U>
__device__ int wg_normalize(const WG &c, const i64 (&d)[2 * U], u64 (&y)[U], int l, bool canon,
                            i64 *sh, u64 *scr)
{
    u64 lo[U];
    i64 hi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        i128 v = (i128)d[2 * u] + (i128)d[2 * u + 1] * ((i128)1 << 32);
        lo[u] = (u64)v;
        hi[u] = (i64)(v >> 64);
        if (m < l) sh[m] = hi[u];
    }
    __syncthreads();
    const i64 hl = sh[l - 1];
    int cc[U];
    u64 f[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        f[u] = 0;
        cc[u] = 0;
        if (m < l) {
            i64 hp = m ? sh[m - 1] : -hl;  // the top limb's overflow wraps negated
            i128 e = (i128)lo[u] + hp;
            f[u] = (u64)e;
            cc[u] = (int)(i64)(e >> 64);  // in {-1, 0, 1}
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) sh[m] = cc[u];
    }
    __syncthreads();
    int top = (int)sh[l - 1];  // carry out of the top limb stays in the carry limb
    u32 inc = 0, dec = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m > 0 && m < l) {
            i64 cm = sh[m - 1];
            inc |= (u32)(cm == 1) << u;
            dec |= (u32)(cm == -1) << u;
        }
    }
    // f + inc (binary carries)
    u32 gm = 0, pm = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        u32 in = (inc >> u) & 1;
        if (m < l) {
            gm |= (u32)(in && f[u] == MPF_MAXL) << u;
            pm |= (u32)(in ? (f[u] == MPF_MAXL - 1) : (f[u] == MPF_MAXL)) << u;
        } else {
            pm |= 1u << u;
        }
    }
    u32 co;
    u32 ci = wg_scan<U>(c, gm, pm, 0, &co, scr);
#pragma unroll
    for (int u = 0; u < U; ++u) f[u] += ((inc >> u) & 1) + ((ci >> u) & 1);
    top += (int)co;
    // f - dec (binary borrows)
    gm = 0;
    pm = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        u32 dn = (dec >> u) & 1;
        if (m < l) {
            gm |= (u32)(dn && f[u] == 0) << u;
            pm |= (u32)(dn ? (f[u] == 1) : (f[u] == 0)) << u;
        } else {
            pm |= 1u << u;
        }
    }
    ci = wg_scan<U>(c, gm, pm, 0, &co, scr);
#pragma unroll
    for (int u = 0; u < U; ++u) f[u] -= ((dec >> u) & 1) + ((ci >> u) & 1);
    top -= (int)co;

    if (canon && top != 0) {  // top is workgroup-uniform
        // value == f - top with f in [0, 2^N), |top| <= 2
        const bool sub = top > 0;
        const u64 s = (u64)(sub ? top : -top);
        gm = 0;
        pm = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            if (m >= l) {
                pm |= 1u << u;
            } else if (m == 0) {
                if (sub) {
                    gm |= (u32)(f[u] < s) << u;
                    pm |= (u32)(f[u] == s) << u;
                } else {
                    u64 t2;
                    gm |= (u32)add_ovf(f[u], s, &t2) << u;
                    pm |= (u32)(t2 == MPF_MAXL) << u;
                }
            } else {
                pm |= (u32)(sub ? (f[u] == 0) : (f[u] == MPF_MAXL)) << u;
            }
        }
        ci = wg_scan<U>(c, gm, pm, 0, &co, scr);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            u64 add = (m == 0 ? s : 0) + ((ci >> u) & 1);
            f[u] = sub ? f[u] - add : f[u] + add;
        }
        top = 0;
        if (co) {
            // sub: f = 2^N + y - top >= 2^N - 2, true value f + 1.
            // add: f = y + |top| - 2^N in {0, 1}, true value f - 1.
            if (c.t == 0) sh[0] = (i64)f[0];
            __syncthreads();
            const u64 f0 = (u64)sh[0];
            const bool to_2N = sub ? (f0 == MPF_MAXL) : (f0 == 0);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int m = u * c.nt + c.t;
                if (to_2N) f[u] = 0;
                else if (m == 0) f[u] = sub ? f[u] + 1 : f[u] - 1;
            }
            top = to_2N ? 1 : 0;
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = f[u];
    __syncthreads();
    return top;
}

// ---------------------------------------------------------------------------
// Multiplication by 2^e mod p in carry-save digits (the FFT twiddle,
// FFT_twiddle mul_fft.c:926 / the butterfly shifts :553-752):
//   2^e = (-1)^neg * 2^(32 y + b);  digit j of the result takes the low 32 bits
//   of (d_{j-y} << b) and the high part of d_{j-y-1} << b, each negated when
//   its source wrapped past 2^N.  |result| < 2^33 + |d|/2: never grows the
//   digit bound, so the rotation can run at every level of a pass.
// ---------------------------------------------------------------------------
struct Rot {
    int y;       // whole digits
    int b;       // bits, 0..31
    i64 sgn;     // +1 / -1
};

__device__ __forceinline__ Rot make_rot(u64 e, u64 N)
{
    Rot r;
    e %= 2 * N;
    r.sgn = 1;
    if (e >= N) { r.sgn = -1; e -= N; }
    r.y = (int)(e >> 5);
    r.b = (int)(e & 31);
    return r;
}

__device__ __forceinline__ i64 rot_digit(const i64 *stage, int j, const Rot &r, int L)
{
    int k0 = j - r.y;
    i64 s0 = 1;
    if (k0 < 0) { k0 += L; s0 = -1; }
    int k1 = j - r.y - 1;
    i64 s1 = 1;
    if (k1 < 0) { k1 += L; s1 = -1; }
    const i64 x0 = stage[k0], x1 = stage[k1];
    const u64 l0 = (u64)(u32)x0 << r.b;
    const u64 l1 = (u64)(u32)x1 << r.b;
    const i64 part0 = (i64)(l0 & MPF_M32);
    const i64 part1 = (i64)(l1 >> 32) + (x1 >> 32) * ((i64)1 << r.b);
    return r.sgn * (s0 * part0 + s1 * part1);
}

// x <- x * 2^e (rot given).  stage: L i64 of LDS private to this call.
// Barrier before (stage free) is the caller's; this function syncs after
// writing and leaves the reads un-fenced (caller syncs before reusing stage).
template <int U>
__device__ __forceinline__ void rot_write(const WG &c, const i64 (&x)[2 * U], i64 *stage, int l)
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) {
            stage[2 * m] = x[2 * u];
            stage[2 * m + 1] = x[2 * u + 1];
        }
    }
}

template <int U>
__device__ __forceinline__ void rot_read(const WG &c, i64 (&x)[2 * U], const i64 *stage, const Rot &r, int l)
{
    const int L = 2 * l;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) {
            x[2 * u] = rot_digit(stage, 2 * m, r, L);
            x[2 * u + 1] = rot_digit(stage, 2 * m + 1, r, L);
        }
    }
}

// full rotation with one staging buffer (two barriers)
template <int U>
__device__ void wg_rotate(const WG &c, i64 (&x)[2 * U], i64 *stage, u64 e, u64 N, int l)
{
    const Rot r = make_rot(e, N);
    rot_write<U>(c, x, stage, l);
    __syncthreads();
    rot_read<U>(c, x, stage, r, l);
    __syncthreads();
}

// ---------------------------------------------------------------------------
// HBM <-> registers
// ---------------------------------------------------------------------------
template <int U>
__device__ __forceinline__ void load_coeff(const WG &c, i64 (&d)[2 * U], const u64 *dig, const int *top,
                                           long slot, int l)
{
    const u64 *p = dig + (size_t)slot * (size_t)l;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        u64 v = (m < l) ? p[m] : 0;
        d[2 * u] = (i64)(v & MPF_M32);
        d[2 * u + 1] = (i64)(v >> 32);
    }
    if (c.t == 0) d[0] -= top[slot];  // top * 2^N == -top
}

template <int U>
__device__ __forceinline__ void zero_coeff(i64 (&d)[2 * U])
{
#pragma unroll
    for (int k = 0; k < 2 * U; ++k) d[k] = 0;
}

// Fused split (FFT_split_bits, mul_fft.c:115-170): coefficient j is the bits1-bit
// chunk at bit offset j*bits1 of the operand (bits past its end read as 0).
template <int U>
__device__ __forceinline__ void load_split(const WG &c, i64 (&d)[2 * U], const u64 *src, long nsrc,
                                           long j, u64 bits1, int l)
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        u64 v = 0;
        if (m < l && (u64)m * 64 < bits1) {
            u64 off = (u64)j * bits1 + (u64)m * 64;
            long q = (long)(off >> 6);
            int s = (int)(off & 63);
            u64 w0 = (q < nsrc) ? src[q] : 0;
            u64 w1 = (s && q + 1 < nsrc) ? src[q + 1] : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
            u64 left = bits1 - (u64)m * 64;
            if (left < 64) v &= (((u64)1) << left) - 1;
        }
        d[2 * u] = (i64)(v & MPF_M32);
        d[2 * u + 1] = (i64)(v >> 32);
    }
}

template <int U>
__device__ __forceinline__ void store_coeff(const WG &c, const u64 (&y)[U], int topv, u64 *dig, int *top,
                                            long slot, int l)
{
    u64 *p = dig + (size_t)slot * (size_t)l;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) p[m] = y[u];
    }
    if (c.t == 0) top[slot] = topv;
}

__device__ __forceinline__ long revbin_dev(long in, int bits)
{
    return bits ? (long)(__brevll((u64)in) >> (64 - bits)) : 0;
}
