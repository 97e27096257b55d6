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
typedef uint8_t u8;

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
// Workgroup carry-lookahead over the l limbs of G independent coefficients.
//   g[gi] (bit u): limb u*nt+t of coefficient gi generates a carry;
//   p[gi] (bit u): it propagates one.  Out: ci[gi] bit u = carry into that limb,
//   co[gi] = carry out of the coefficient's last limb.  Limbs that do not exist
//   must have g = 0, p = 1.
// Lane level: a 64-bit add of the ballot masks (generate = 2, propagate = 1)
// yields every lane's carry in one instruction; entry level (one entry per
// (coefficient, u, wave), U*nw <= 64 entries per coefficient) the same trick in
// wave 0, one 64-lane step per coefficient.  Two barriers regardless of G.
// scr: >= 3*G*U*nw + G u64 of LDS.
// ---------------------------------------------------------------------------
template <int U, int G>
__device__ u32 wg_scan_multi(const WG &c, u32 g, u32 p, u32 *co_mask, u64 *scr)
{
    // bit (gi*U + u) of g / p / result: limb u*nt+t of coefficient gi
    const int EG = U * c.nw;
    const int E = G * EG;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 gmask = __ballot((g >> (gi * U + u)) & 1);
            const u64 pmask = __ballot((p >> (gi * U + u)) & 1);
            if (c.lane == 0) {
                const int e = gi * EG + u * c.nw + c.wave;
                scr[2 * e] = gmask;
                scr[2 * e + 1] = pmask;
            }
        }
    }
    __syncthreads();
    if (c.wave == 0) {
        u32 com = 0;
        for (int gi = 0; gi < G; ++gi) {
            const int e = c.lane;
            bool eg = false, ep = true;
            if (e < EG) {
                const int k = gi * EG + e;
                u64 X = scr[2 * k], Y = X | scr[2 * k + 1], s, s2;
                bool o0 = add_ovf(X, Y, &s);
                bool o1 = o0 | add_ovf(s, 1, &s2);
                eg = o0;
                ep = o1 && !o0;
            }
            u64 X = __ballot(eg), Y = X | __ballot(ep), s;
            bool o = add_ovf(X, Y, &s);
            u64 CI = s ^ X ^ Y;
            if (e < EG) scr[2 * E + gi * EG + e] = (CI >> c.lane) & 1;
            com |= (u32)o << gi;
        }
        if (c.lane == 0) scr[3 * E] = com;
    }
    __syncthreads();
    u32 ci = 0;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = gi * EG + u * c.nw + c.wave;   // masks re-read: keeps them out of VGPRs
            u64 cin = scr[2 * E + e];
            u64 X = scr[2 * e], Y = X | scr[2 * e + 1], s, s2;
            add_ovf(X, Y, &s);
            add_ovf(s, cin, &s2);
            u64 C = s2 ^ X ^ Y;
            ci |= (u32)((C >> c.lane) & 1) << (gi * U + u);
        }
    }
    *co_mask = (u32)scr[3 * E];
    __syncthreads();
    return ci;
}

// single-coefficient scan with a carry-in (used by the combine kernels, U limbs/thread)
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

// LDS needed by wg_norm_multi: edge (int32) and scan scratch (u64)
__host__ __device__ constexpr int norm_edge_ints(int G, int U, int nw) { return G * U * nw + 2 * G + 4; }
__host__ __device__ constexpr int norm_scr_u64(int G, int U, int nw) { return 3 * G * U * nw + 2 * G + 8; }

// value of limb m-1's `v` for the thread owning limb m = u*nt+t (strided ownership):
// lanes 1..63 take lane-1 (DPP), lane 0 reads the previous wave's / previous row's
// last lane from `edge`.  `first` is returned for limb 0.
__device__ __forceinline__ int prev_limb_val(const WG &c, int v, const int *edge_row, const int *edge_prev_row,
                                             int u, int first)
{
    int pv = __shfl_up(v, 1);
    if (c.lane == 0) pv = c.wave ? edge_row[c.wave - 1] : (u ? edge_prev_row[c.nw - 1] : first);
    return pv;
}

// ---------------------------------------------------------------------------
// Resolve carry-save digits of G coefficients into limbs (one pass of barriers
// for all G).
//   d[gi][2u], d[gi][2u+1]: digits 2m, 2m+1 of limb m = u*nt+t (|d| < 2^62).
//   Out: y[gi][u] limbs and top[gi], value = y + top * 2^N (mod p).
//   canon = false: top in [-2, 2] ("reduced", what the next pass reloads).
//   canon = true : canonical residue in [0, 2^N] (top in {0,1}, 1 only for
//                  exactly 2^N) == mpn_normmod_2expp1 (mul_fft.c:272-294).
// Round A/B turn the carry-save digits into 64-bit limbs with carries in
// {-1, 0, 1}; round C resolves those with two binary carry-lookahead scans
// (+1s, then -1s); the carry out of the top limb stays in the carry limb.
// ---------------------------------------------------------------------------
template <int U, int G>
__device__ void wg_norm_multi(const WG &c, const i64 (&d)[G][2 * U], u64 (&y)[G][U], int (&top)[G],
                              int (&cout)[G][U], int l, bool canon, int *edge, u64 *scr)
{
    static_assert(G * U <= 32, "bitmasks hold G*U bits");
    const int EGw = U * c.nw;
    int *elast = edge + G * EGw;  // per coefficient: the value at limb l-1
    u64 f[G][U];
    int cc[G][U];
    {
        int hv[G][U];
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int m = u * c.nt + c.t;
                i128 v = (i128)d[gi][2 * u] + (i128)d[gi][2 * u + 1] * ((i128)1 << 32);
                f[gi][u] = m < l ? (u64)v : 0;
                hv[gi][u] = m < l ? (int)(i64)(v >> 64) : 0;  // |hi| < 2^30
                if (c.lane == 63) edge[gi * EGw + u * c.nw + c.wave] = hv[gi][u];
                if (m == l - 1) elast[gi] = hv[gi][u];
            }
        }
        __syncthreads();
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
            const int *er = edge + gi * EGw;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int m = u * c.nt + c.t;
                // the top limb's overflow wraps negated into limb 0
                const int hp = prev_limb_val(c, hv[gi][u], er + u * c.nw, er + (u - 1) * c.nw, u, -elast[gi]);
                const i128 e = (i128)f[gi][u] + hp;
                f[gi][u] = m < l ? (u64)e : 0;
                cc[gi][u] = m < l ? (int)(i64)(e >> 64) : 0;  // in {-1, 0, 1}
            }
        }
    }
    if (!canon) {
        // "reduced": limbs f plus their carries c in {-1,0,1} (stored as ballot masks by
        // the caller; the next pass folds c_{m-1} into digit 2m) -- no carry chains.
        __syncthreads();  // edge is reused by the caller's next call
#pragma unroll
        for (int gi = 0; gi < G; ++gi)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                y[gi][u] = f[gi][u];
                cout[gi][u] = cc[gi][u];
            }
#pragma unroll
        for (int gi = 0; gi < G; ++gi) top[gi] = 0;
        return;
    }
    __syncthreads();
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = u * c.nt + c.t;
            if (c.lane == 63) edge[gi * EGw + u * c.nw + c.wave] = cc[gi][u];
            if (m == l - 1) elast[gi] = cc[gi][u];
        }
    }
    __syncthreads();
    u32 inc = 0, dec = 0, gm = 0, pm = 0, ci, com;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int *er = edge + gi * EGw;
        top[gi] = elast[gi];  // carry out of the top limb stays in the carry limb
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = u * c.nt + c.t;
            const int b = gi * U + u;
            const int cm = prev_limb_val(c, cc[gi][u], er + u * c.nw, er + (u - 1) * c.nw, u, 0);
            if (m > 0 && m < l) {
                inc |= (u32)(cm == 1) << b;
                dec |= (u32)(cm == -1) << b;
            }
            // f + inc (binary carries)
            const u32 in = (inc >> b) & 1;
            if (m < l) {
                gm |= (u32)(in && f[gi][u] == MPF_MAXL) << b;
                pm |= (u32)(in ? (f[gi][u] == MPF_MAXL - 1) : (f[gi][u] == MPF_MAXL)) << b;
            } else {
                pm |= 1u << b;
            }
        }
    }
    ci = wg_scan_multi<U, G>(c, gm, pm, &com, scr);
    gm = pm = 0;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        top[gi] += (int)((com >> gi) & 1);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = u * c.nt + c.t;
            const int b = gi * U + u;
            f[gi][u] += ((inc >> b) & 1) + ((ci >> b) & 1);
            // f - dec (binary borrows)
            const u32 dn = (dec >> b) & 1;
            if (m < l) {
                gm |= (u32)(dn && f[gi][u] == 0) << b;
                pm |= (u32)(dn ? (f[gi][u] == 1) : (f[gi][u] == 0)) << b;
            } else {
                pm |= 1u << b;
            }
        }
    }
    ci = wg_scan_multi<U, G>(c, gm, pm, &com, scr);
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        top[gi] -= (int)((com >> gi) & 1);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int b = gi * U + u;
            f[gi][u] -= ((dec >> b) & 1) + ((ci >> b) & 1);
        }
    }

    if (canon) {
        bool any = false;
#pragma unroll
        for (int gi = 0; gi < G; ++gi) any |= top[gi] != 0;  // workgroup-uniform
        if (any) {
            // value == f - top, f in [0, 2^N), |top| <= 2: one more carry/borrow chain
            gm = pm = 0;
#pragma unroll
            for (int gi = 0; gi < G; ++gi) {
                const bool sub = top[gi] > 0;
                const u64 sv = (u64)(sub ? top[gi] : -top[gi]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int m = u * c.nt + c.t;
                    const int b = gi * U + u;
                    if (m >= l) {
                        pm |= 1u << b;
                    } else if (m == 0) {
                        if (sub) {
                            gm |= (u32)(f[gi][u] < sv) << b;
                            pm |= (u32)(f[gi][u] == sv) << b;
                        } else {
                            u64 t2;
                            gm |= (u32)add_ovf(f[gi][u], sv, &t2) << b;
                            pm |= (u32)(t2 == MPF_MAXL) << b;
                        }
                    } else {
                        pm |= (u32)(sub ? (f[gi][u] == 0) : (f[gi][u] == MPF_MAXL)) << b;
                    }
                }
            }
            ci = wg_scan_multi<U, G>(c, gm, pm, &com, scr);
            u64 *f0 = scr;  // the scan left scr free
#pragma unroll
            for (int gi = 0; gi < G; ++gi) {
                const bool sub = top[gi] > 0;
                const u64 sv = (u64)(sub ? top[gi] : -top[gi]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int m = u * c.nt + c.t;
                    const u64 add = (m == 0 ? sv : 0) + ((ci >> (gi * U + u)) & 1);
                    f[gi][u] = sub ? f[gi][u] - add : f[gi][u] + add;
                }
                if (c.t == 0) f0[gi] = f[gi][0];
            }
            __syncthreads();
#pragma unroll
            for (int gi = 0; gi < G; ++gi) {
                const bool sub = top[gi] > 0;
                if (top[gi] != 0 && ((com >> gi) & 1)) {
                    // sub: f = 2^N + y - top >= 2^N - 2, true value f + 1.
                    // add: f = y + |top| - 2^N in {0, 1}, true value f - 1.
                    const bool to_2N = sub ? (f0[gi] == MPF_MAXL) : (f0[gi] == 0);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int m = u * c.nt + c.t;
                        if (to_2N) f[gi][u] = 0;
                        else if (m == 0) f[gi][u] = sub ? f[gi][u] + 1 : f[gi][u] - 1;
                    }
                    top[gi] = to_2N ? 1 : 0;
                } else {
                    top[gi] = 0;
                }
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            y[gi][u] = f[gi][u];
            cout[gi][u] = 0;
        }
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

// e must already be reduced into [0, 2N) (2N < 2^20 for every supported size)
__device__ __forceinline__ Rot make_rot(u64 e, u64 N)
{
    Rot r;
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
    const i64 part1 = (i64)(l1 >> 32) + (i64)((u64)(x1 >> 32) << r.b);  // two's complement shift == * 2^b
    return r.sgn * (s0 * part0 + s1 * part1);
}

// x <- x * 2^e (rot given).  stage: L i64 of LDS private to this call.
// Barrier before (stage free) is the caller's; this function syncs after
// writing and leaves the reads un-fenced (caller syncs before reusing stage).
template <int U>
__device__ __forceinline__ void rot_write(const WG &c, const i64 (&x)[2 * U], i64 *stage, int l)
{
    typedef long long v2i __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) {
            v2i v;
            v.x = x[2 * u];
            v.y = x[2 * u + 1];
            *(v2i *)(stage + 2 * m) = v;   // one ds_write_b128 per limb
        }
    }
}

template <int U>
__device__ __forceinline__ void rot_read(const WG &c, i64 (&x)[2 * U], const i64 *stage, const Rot &r, int l)
{
    const int L = 2 * l;
    if (r.b == 0 && !(r.y & 1)) {
        // limb-aligned shift (every FFT twiddle when w*NC and w*NR are multiples of 64):
        // a signed limb permutation, one 16-byte LDS read per limb
        typedef long long v2i __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = u * c.nt + c.t;
            if (m < l) {
                int k = 2 * m - r.y;
                i64 sg = r.sgn;
                if (k < 0) { k += L; sg = -sg; }
                const v2i v = *(const v2i *)(stage + k);
                x[2 * u] = sg * v.x;
                x[2 * u + 1] = sg * v.y;
            }
        }
        return;
    }
    if (r.b == 0) {   // digit-aligned: signed digit permutation
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = u * c.nt + c.t;
            if (m < l) {
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    int k = 2 * m + v - r.y;
                    i64 sg = r.sgn;
                    if (k < 0) { k += L; sg = -sg; }
                    x[2 * u + v] = sg * stage[k];
                }
            }
        }
        return;
    }
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
// One operand's coefficient store in HBM (DESIGN.md "Data layout").
//   dig[slot*l + m]   limb m
//   cb[slot*cbw + 2W] / [.. + 1]: bit k set = limb 64W+k carries +1 / -1 into limb 64W+k+1
//                     ("reduced" form written by intermediate passes; zero when canonical)
//   top[slot]         carry limb: value = limbs + carries + top * 2^N
struct Coef {
    u64 *dig;
    u64 *cb;
    int *top;
};

__host__ __device__ inline int cb_words(int l) { return 2 * ((l + 63) / 64); }

template <int U>
__device__ __forceinline__ void load_coeff(const WG &c, i64 (&d)[2 * U], const Coef &s, long slot, int l)
{
    const u64 *p = s.dig + (size_t)slot * (size_t)l;
    const int cbw = cb_words(l);
    const u64 *cbp = s.cb + (size_t)slot * (size_t)cbw;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = u * c.nt + c.t;
        u64 v = 0;
        i64 cin = 0;
        if (m < l) {
            v = p[m];
            const int W = m >> 6;             // = u*nw + wave: wave-uniform
            const u64 pw = cbp[2 * W], nwm = cbp[2 * W + 1];
            if (c.lane) {
                cin = (i64)((pw >> (c.lane - 1)) & 1) - (i64)((nwm >> (c.lane - 1)) & 1);
            } else if (W) {
                cin = (i64)(cbp[2 * W - 2] >> 63) - (i64)(cbp[2 * W - 1] >> 63);
            }
        }
        d[2 * u] = (i64)(v & MPF_M32) + cin;
        d[2 * u + 1] = (i64)(v >> 32);
    }
    if (c.t == 0) {
        // carry limb plus the reduced form's carry out of limb l-1: both weigh 2^N == -1
        const int W = (l - 1) >> 6, b = (l - 1) & 63;
        const i64 cl = (i64)((cbp[2 * W] >> b) & 1) - (i64)((cbp[2 * W + 1] >> b) & 1);
        d[0] -= s.top[slot] + cl;
    }
}

template <int U>
__device__ __forceinline__ void zero_coeff(i64 (&d)[2 * U])
{
#pragma unroll
    for (int k = 0; k < 2 * U; ++k) d[k] = 0;
}

// Where the fused split reads the operand: the whole operand (chunk == 0), or one rank's
// column slice of it (multi-GPU, sharded.py): for every MFA position p the limbs from
// floor((p NC + c0) bits1 / 64) on, `chunk` of them per position, back to back.
struct SrcSlice {
    long chunk;   // limbs per position, 0 = whole operand
    long NC;      // columns (a power of two)
    long c0;      // first column of the slice
};

// limb q of the operand as seen by coefficient j = p NC + c (bits past its end read as 0)
__device__ __forceinline__ u64 src_limb(const u64 *src, long nsrc, const SrcSlice &v, long j, u64 bits1, long q)
{
    if (q >= nsrc) return 0;
    if (!v.chunk) return src[q];
    const long p = j >> __builtin_ctzl((unsigned long)v.NC);
    const long r = q - (long)(((u64)(p * v.NC + v.c0) * bits1) >> 6);   // >= 0 for the slice's coefficients
    return r < v.chunk ? src[p * v.chunk + r] : 0;
}

// Fused split (FFT_split_bits, mul_fft.c:115-170): coefficient j is the bits1-bit
// chunk at bit offset j*bits1 of the operand (bits past its end read as 0).
template <int U>
__device__ __forceinline__ void load_split(const WG &c, i64 (&d)[2 * U], const u64 *src, long nsrc,
                                           const SrcSlice &sv, long j, u64 bits1, int l)
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        u64 v = 0;
        if (m < l && (u64)m * 64 < bits1) {
            u64 off = (u64)j * bits1 + (u64)m * 64;
            long q = (long)(off >> 6);
            int s = (int)(off & 63);
            u64 w0 = src_limb(src, nsrc, sv, j, bits1, q);
            u64 w1 = s ? src_limb(src, nsrc, sv, j, bits1, q + 1) : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
            u64 left = bits1 - (u64)m * 64;
            if (left < 64) v &= (((u64)1) << left) - 1;
        }
        d[2 * u] = (i64)(v & MPF_M32);
        d[2 * u + 1] = (i64)(v >> 32);
    }
}

template <int U>
__device__ __forceinline__ void store_coeff(const WG &c, const u64 (&y)[U], const int (&cy)[U], int topv,
                                            const Coef &s, long slot, int l)
{
    u64 *p = s.dig + (size_t)slot * (size_t)l;
    const int cbw = cb_words(l);
    u64 *cbp = s.cb + (size_t)slot * (size_t)cbw;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int m = u * c.nt + c.t;
        if (m < l) p[m] = y[u];
        const u64 pm = __ballot(m < l && cy[u] == 1);
        const u64 nm = __ballot(m < l && cy[u] == -1);
        const int W = (u * c.nt + c.wave * 64) >> 6;
        if (c.lane == 0 && 2 * W < cbw) {
            cbp[2 * W] = pm;
            cbp[2 * W + 1] = nm;
        }
    }
    if (c.t == 0) s.top[slot] = topv;
}

__device__ __forceinline__ long revbin_dev(long in, int bits)
{
    return bits ? (long)(__brevll((u64)in) >> (64 - bits)) : 0;
}
