// lkernels.hpp -- LDS-resident radix-2^LOGG passes for small coefficients
// (l <= 256 limbs: G = 2^LOGG coefficients of 2l carry-save digits fit in LDS).
//
// One workgroup = G/2 waves owns one butterfly group of G coefficients for LOGG
// levels (FFT_radix2_twiddle / FFT_radix2 / IFFT_radix2(_twiddle), mul_fft.c:1397,
// :786, :1444, :1964).  The coefficients live in LDS between levels; at every level
// wave q reads its butterfly pair, adds/subtracts, and writes both results back in
// place, so one barrier per level suffices (no slot is touched by two waves within
// a level).  Every multiplication by 2^e is deferred into the NEXT read of that slot
// as a "pending exponent" -- a rotation is only an index permutation (with sign and
// sub-digit shift) of the LDS read (wv_rot_read), and exponents of successive
// rotations simply add mod 2N.  So the MFA twiddles (README:89), the DIF output
// twiddles, the DIT input twiddles and the final 2^-(depth+1) scaling
// (mul_fft.c:3256-3260) cost no extra LDS round trip.
// Load/store and carry resolution are the wave-owned routines of wave.hpp: wave q
// loads and stores coefficients 2q and 2q+1.
#pragma once
#include "wkernels.hpp"

// pending exponent of slot k after forward (DIF) level LI: 2^(e0 + (k mod 2^JB) estep)
// for the difference output of each pair (bit JB of k set), 0 for the sum
template <int LOGG, int DIR, int LI>
__device__ __forceinline__ u64 lp_level_exp(const PassArgs &a, int pos0, int pstep, int k)
{
    constexpr int JB = DIR == 0 ? LOGG - 1 - LI : LI;
    if (!((k >> JB) & 1)) return 0;
    const int level = DIR == 0 ? a.lvl0 + LI : a.lvl0 + LOGG - 1 - LI;
    const int h = 1 << (a.lbM - level - 1);
    const u64 unit = a.rho << level;
    return (u64)(pos0 & (h - 1)) * unit + (u64)(k & ((1 << JB) - 1)) * (u64)pstep * unit;
}

__device__ __forceinline__ u64 lp_add(u64 e, u64 f, u64 N2)
{
    const u64 s = e + f;
    return s >= N2 ? s - N2 : s;
}

// x <- slot * 2^E (E in [0, 2N))
template <int U, bool F>
__device__ __forceinline__ void lp_read(i64 (&x)[2 * U], const i64 *slot, u64 E, u64 N, int l, int lane)
{
    typedef long long v2i __attribute__((ext_vector_type(2)));
    if (E == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = 64 * u + lane;
            if (wv_in<F>(m, l)) {
                const v2i v = *(const v2i *)(slot + 2 * m);
                x[2 * u] = v.x;
                x[2 * u + 1] = v.y;
            } else {
                x[2 * u] = x[2 * u + 1] = 0;
            }
        }
    } else {
        wv_rot_read<U, F>(x, slot, make_rot(E, N), l, lane);
    }
}

// the LI-th level: wave q handles pair (i, k = i | 2^JB), i = q with a zero inserted at bit JB
template <int U, bool F, int LOGG, int DIR, int LI>
__device__ __forceinline__ void lp_levels(i64 *lds, const PassArgs &a, int pos0, int pstep, u64 tw0, u64 twst, int q,
                                          int lane)
{
    constexpr int JB = DIR == 0 ? LOGG - 1 - LI : LI;
    const int l = a.l;
    const u64 N2 = 2 * a.N;
    const int i = ((q >> JB) << (JB + 1)) | (q & ((1 << JB) - 1));
    const int k = i | (1 << JB);
    // what the previous step left pending on slots i and k
    u64 pi = 0, pk = 0;
    if constexpr (LI == 0) {
        if (a.tw_mode == 1) {
            pi = tw0 + (u64)i * twst;
            pk = tw0 + (u64)k * twst;
        }
    } else if constexpr (DIR == 0) {
        pi = lp_level_exp<LOGG, DIR, LI - 1>(a, pos0, pstep, i);
        pk = lp_level_exp<LOGG, DIR, LI - 1>(a, pos0, pstep, k);
    }
    if (DIR == 1) {   // DIT: t = 2^-e x_k, then (x_i + t, x_i - t)
        const u64 e = lp_level_exp<LOGG, DIR, LI>(a, pos0, pstep, k);
        pk = lp_add(pk, e ? N2 - e : 0, N2);
    }
    i64 *si = lds + (size_t)i * 2 * l, *sk = lds + (size_t)k * 2 * l;
    i64 xi[2 * U], xk[2 * U];
    lp_read<U, F>(xi, si, pi, a.N, l, lane);
    lp_read<U, F>(xk, sk, pk, a.N, l, lane);
#pragma unroll
    for (int t = 0; t < 2 * U; ++t) {
        const i64 s = xi[t] + xk[t], d = xi[t] - xk[t];
        xi[t] = s;
        xk[t] = d;
    }
    wv_rot_write<U, F>(xi, si, l, lane);
    wv_rot_write<U, F>(xk, sk, l, lane);   // DIF: its output twiddle stays pending
    __syncthreads();
    if constexpr (LI + 1 < LOGG) lp_levels<U, F, LOGG, DIR, LI + 1>(lds, a, pos0, pstep, tw0, twst, q, lane);
}

template <int U, bool F, int LOGG, int DIR>
__global__ __launch_bounds__(32 << LOGG) void k_lpass(PassArgs a)
{
    pass_clear_flags(a);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    i64 *lds = (i64 *)smem;
    const int lane = wv_lane();
    const int q = wv_id();   // wave = pair index
    const int l = a.l;
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
    const u64 N2 = 2 * a.N;
    const int pos0 = bstart | lo;
    const int pstep = 1 << lobits;
    const long sbase = (long)sub * a.sub_stride;
    auto slot_of = [&](int i) -> long {
        const int ps = a.pos_off + pos0 + i * pstep;
        return sbase + (long)(ps >> a.pbb) * a.pbs + (long)(ps & ((1 << a.pbb) - 1)) * a.pos_stride;
    };
    const u64 rsub = a.tw_mode ? (u64)revbin_dev(a.sub_off + sub, a.tw_lbR) : 0;
    const u64 tw0 = a.tw_w * (u64)(a.pos_off + pos0) * rsub, twst = a.tw_w * (u64)pstep * rsub;

    // ---- load: wave q brings coefficients 2q, 2q+1 into LDS ------------------------
    {
        i64 x[2][2 * U];
        if (a.src[op]) {   // first forward column pass: split fused into the load
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int i = 2 * q + c;
                if (DIR == 0 && pos0 + i * pstep >= a.zero_from) zero_coeff<U>(x[c]);
                else wv_load_split<U, F>(x[c], a.src[op], a.nsrc[op], SrcSlice{a.src_chunk, a.jNC, a.sub_off},
                                         (long)(a.pos_off + pos0 + i * pstep) * a.jNC + a.sub_off + sub, a.bits1, l,
                                         lane);
            }
        } else {
            WvRaw<U> raw[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int i = 2 * q + c;
                if (!(DIR == 0 && pos0 + i * pstep >= a.zero_from)) wv_load_raw<U, F>(raw[c], st, slot_of(i), l, lane);
            }
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int i = 2 * q + c;
                if (DIR == 0 && pos0 + i * pstep >= a.zero_from) zero_coeff<U>(x[c]);
                else wv_load_digits<U, F>(x[c], raw[c], l, lane);
            }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) wv_rot_write<U, F>(x[c], lds + (size_t)(2 * q + c) * 2 * l, l, lane);
    }
    __syncthreads();

    lp_levels<U, F, LOGG, DIR, 0>(lds, a, pos0, pstep, tw0, twst, q, lane);

    // ---- store: wave q normalises coefficients 2q, 2q+1 -----------------------------
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int i = 2 * q + c;
        u64 e = 0;
        if (DIR == 0) {
            e = lp_level_exp<LOGG, DIR, LOGG - 1>(a, pos0, pstep, i);
        } else {
            if (a.tw_mode == 2) {
                const u64 t = tw0 + (u64)i * twst;
                e = t ? N2 - t : 0;
            }
            if (a.scale_e) e = lp_add(e, a.scale_e, N2);
        }
        const int bs = (pos0 + i * pstep) & ~(pstep - 1);
        const bool keep = DIR == 1 || (bs < a.need && bs + pstep > a.need_lo);
        if (keep) {
            i64 x[2 * U];
            lp_read<U, F>(x, lds + (size_t)i * 2 * l, e, a.N, l, lane);
            wv_normalize_store<U, F>(x, a.canon != 0, st, slot_of(i), l, lane);
        }
    }
}
