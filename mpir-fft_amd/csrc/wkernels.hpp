// wkernels.hpp -- wave-owned coefficient kernels (64 (U-1) < l <= 64 U limbs, U in 1..4;
// F: l == 64 U).
//
// Same work and HBM format as k_pass / k_pairop / k_scale (kernels.hpp), but every
// wavefront owns its G coefficients outright: no workgroup barriers, carries
// resolved with DPP + ballots (wave.hpp).  A workgroup is just WPB independent waves
// sharing a launch; each wave has its own LDS staging buffer.
//   k_wpass<U,LOGG,DIR>  forward DIF / inverse DIT radix-2^LOGG pass
//                        (FFT_radix2_twiddle / FFT_radix2 / IFFT_radix2(_twiddle),
//                        mul_fft.c:1397, :786, :1444, :1964; MFA twiddles README:89;
//                        fused split mul_fft.c:115), optional fused scale
//                        (mul_fft.c:3256-3260)
//   k_wpair<U>           element-wise steps of the truncated inverse
//                        (IFFT_radix2_truncate(1)_twiddle, mul_fft.c:1604, :1733)
//   k_wscale<U>          2^-(depth+1) scaling + normmod (mul_fft.c:3256-3260)
#pragma once
#include "kernels.hpp"
#include "wave.hpp"
#include "wdispatch.hpp"

__device__ __forceinline__ int wv_lane() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int wv_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// one radix-2 level of a pass (compile-time level index LI: every register index static)
template <int U, bool F, int LOGG, int DIR, int LI>
__device__ __forceinline__ void wv_levels(i64 (&x)[1 << LOGG][2 * U], const PassArgs &a, int pos0, int pstep,
                                          i64 *stage, int lane)
{
    constexpr int G = 1 << LOGG;
    constexpr int NS = wv_stage_slots(G, U);
    constexpr int JB = DIR == 0 ? LOGG - 1 - LI : LI;   // window bit of the butterfly partner
    const int l = a.l;
    const u64 N2 = 2 * a.N;
    const int level = DIR == 0 ? a.lvl0 + LI : a.lvl0 + LOGG - 1 - LI;
    const int h = 1 << (a.lbM - level - 1);
    const u64 unit = a.rho << level;
    const u64 e0 = (u64)(pos0 & (h - 1)) * unit;
    const u64 estep = (u64)pstep * unit;
    auto sel = [](int k) { return ((k >> JB) & 1) != 0; };
    auto slot = [](int k) { return ((k >> (JB + 1)) << JB) | (k & ((1 << JB) - 1)); };
    if (DIR == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if ((i >> JB) & 1) continue;
            const int k = i | (1 << JB);
#pragma unroll
            for (int q = 0; q < 2 * U; ++q) {
                const i64 s = x[i][q] + x[k][q], d = x[i][q] - x[k][q];
                x[i][q] = s;
                x[k][q] = d;
            }
        }
        wv_rot_rounds<U, F, G, NS, 0>(x, sel, slot, [&](int k) -> u64 {
            return e0 + (u64)(k & ((1 << JB) - 1)) * estep; }, a.N, l, stage, lane);
    } else {
        wv_rot_rounds<U, F, G, NS, 0>(x, sel, slot, [&](int k) -> u64 {
            const u64 e = e0 + (u64)(k & ((1 << JB) - 1)) * estep;
            return e ? N2 - e : 0; }, a.N, l, stage, lane);
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if ((i >> JB) & 1) continue;
            const int k = i | (1 << JB);
#pragma unroll
            for (int q = 0; q < 2 * U; ++q) {
                const i64 s = x[i][q] + x[k][q], d = x[i][q] - x[k][q];
                x[i][q] = s;
                x[k][q] = d;
            }
        }
    }
    if constexpr (LI + 1 < LOGG) wv_levels<U, F, LOGG, DIR, LI + 1>(x, a, pos0, pstep, stage, lane);
}

template <int U, bool F, int LOGG, int DIR>
__global__ __launch_bounds__(64 * WPB) void k_wpass(PassArgs a)
{
    pass_clear_flags(a);
    constexpr int G = 1 << LOGG;
    constexpr int NS = wv_stage_slots(G, U);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = wv_lane();
    const int wv = wv_id();
    const int l = a.l;
    i64 *stage = (i64 *)smem + (size_t)wv * NS * 2 * l;
    const long gw = (long)blockIdx.x * WPB + wv;
    if (gw >= (long)a.nsub * a.ngroups) return;
    const int op = blockIdx.y;
    Coef st;
    st.dig = a.dig[op];
    st.cb = a.cb[op];
    st.top = a.top[op];
    const int sub = (int)(gw / a.ngroups);
    const int grp = (int)(a.grp0 + gw % a.ngroups);
    const int lobits = a.lbM - a.lvl0 - LOGG;
    const int lo = grp & ((1 << lobits) - 1);
    const int hi = grp >> lobits;
    const int bstart = hi << (a.lbM - a.lvl0);
    if (DIR == 0 && (bstart >= a.need || bstart + (1 << (a.lbM - a.lvl0)) <= a.need_lo)) return;   // whole block past the truncation point / outside the rows needed
    const u64 N2 = 2 * a.N;
    const int pos0 = bstart | lo;
    const int pstep = 1 << lobits;
    const long sbase = (long)sub * a.sub_stride;
    auto slot_of = [&](int i) -> long {
        const int ps = a.pos_off + pos0 + i * pstep;
        return sbase + (long)(ps >> a.pbb) * a.pbs + (long)(ps & ((1 << a.pbb) - 1)) * a.pos_stride;
    };

    i64 x[G][2 * U];
    if (a.ablate >= 3) {   // timing experiments only: raw limb copy (3), without the carry data (4)
        u64 v[G][U];
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const long sl = wv_uniform(slot_of(i));
#pragma unroll
            for (int u = 0; u < U; ++u) v[i][u] = st.dig[sl * l + 64 * u + lane];
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const long sl = wv_uniform(slot_of(i));
            if (a.ablate == 3) {
                int cc[U];
#pragma unroll
                for (int u = 0; u < U; ++u) cc[u] = 0;
                wv_store<U, F>(v[i], cc, 0, st, sl, l, lane);
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) st.dig[sl * l + 64 * u + lane] = v[i][u] + 1;
            }
        }
        return;
    }
    if (a.src[op]) {   // first forward column pass: split fused into the load
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if (DIR == 0 && pos0 + i * pstep >= a.zero_from) zero_coeff<U>(x[i]);
            else wv_load_split<U, F>(x[i], a.src[op], a.nsrc[op], SrcSlice{a.src_chunk, a.jNC, a.sub_off},
                                     (long)(a.pos_off + pos0 + i * pstep) * a.jNC + a.sub_off + sub, a.bits1, l, lane);
        }
    } else {
        WvRaw<U> raw[G];
#pragma unroll
        for (int i = 0; i < G; ++i)
            if (!(DIR == 0 && pos0 + i * pstep >= a.zero_from)) wv_load_raw<U, F>(raw[i], st, slot_of(i), l, lane);
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if (DIR == 0 && pos0 + i * pstep >= a.zero_from) zero_coeff<U>(x[i]);
            else wv_load_digits<U, F>(x[i], raw[i], l, lane);
        }
    }

    // MFA twiddles: 2^(tw_w * (pos_off + pos) * revbin(row)), always < 2N
    const u64 rsub = a.tw_mode ? (u64)revbin_dev(a.sub_off + sub, a.tw_lbR) : 0;
    const u64 tw0 = a.tw_w * (u64)(a.pos_off + pos0) * rsub, twst = a.tw_w * (u64)pstep * rsub;
    if (a.ablate) {   // timing experiments only
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if (a.ablate == 2) {
                u64 f[U];
                int cc[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    f[u] = (u64)x[i][2 * u] + ((u64)x[i][2 * u + 1] << 32);
                    cc[u] = 0;
                }
                wv_store<U, F>(f, cc, 0, st, slot_of(i), l, lane);
            } else {
                wv_normalize_store<U, F>(x[i], a.canon != 0, st, slot_of(i), l, lane);
            }
        }
        return;
    }
    if (a.tw_mode == 1)
        wv_rot_all<U, F, G, NS, 0>(x, [&](int i) { return tw0 + (u64)i * twst; }, a.N, l, stage, lane);

    wv_levels<U, F, LOGG, DIR, 0>(x, a, pos0, pstep, stage, lane);

    if (a.tw_mode == 2)
        wv_rot_all<U, F, G, NS, 0>(x, [&](int i) -> u64 {
            const u64 e = tw0 + (u64)i * twst;
            return e ? N2 - e : 0; }, a.N, l, stage, lane);
    if (a.scale_e)   // fused final scaling (whole inverse column transform in this pass)
        wv_rot_all<U, F, G, NS, 0>(x, [&](int) -> u64 { return a.scale_e; }, a.N, l, stage, lane);

#pragma unroll
    for (int i = 0; i < G; ++i) {
        const int bs = (pos0 + i * pstep) & ~(pstep - 1);
        const bool keep = DIR == 1 || (bs < a.need && bs + pstep > a.need_lo);
        if (keep) wv_normalize_store<U, F>(x[i], a.canon != 0, st, slot_of(i), l, lane);
    }
}

// element-wise steps of the truncated inverse column transform (one wave per pair)
template <int U, bool F>
__global__ __launch_bounds__(64 * WPB) void k_wpair(PairArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = wv_lane();
    const int wv = wv_id();
    const int l = a.l;
    i64 *stage = (i64 *)smem + (size_t)wv * 2 * l;
    const long gw = (long)blockIdx.x * WPB + wv;
    if (gw >= (long)a.cnt * a.ncol) return;
    const int col = (int)(gw % a.ncol);
    const int i = a.i0 + (int)(gw / a.ncol);
    long slot[2];
    slot[0] = (long)(a.off + i) * a.NC + col;
    slot[1] = (long)(a.off + i + a.h) * a.NC + col;
    const u64 N2 = 2 * a.N;
    const u64 e = (u32)((u64)i * a.rho) % (u32)N2;
    i64 x[2][2 * U];
    bool keep[2] = {true, false};
    Coef st;
    st.dig = a.dig;
    st.cb = a.cb;
    st.top = a.top;
    wv_load<U, F>(x[0], st, slot[0], l, lane);
    if (a.op != OP_DOUBLE && a.op != OP_FILL) wv_load<U, F>(x[1], st, slot[1], l, lane);
    else zero_coeff<U>(x[1]);
    auto only = [](int which) { return [which](int k) { return k == which; }; };
    auto slot0 = [](int) { return 0; };
    switch (a.op) {
    case OP_DOUBLE:
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) x[0][q] *= 2;
        break;
    case OP_HALFADD:  // a = (a + b) / 2
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) x[0][q] += x[1][q];
        wv_rot_set<U, F, 2>(x, only(0), slot0, [&](int) -> u64 { return N2 - 1; }, a.N, l, stage, lane);
        break;
    case OP_FILL:     // b = 2^e a
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) x[1][q] = x[0][q];
        wv_rot_set<U, F, 2>(x, only(1), slot0, [&](int) -> u64 { return e; }, a.N, l, stage, lane);
        keep[0] = false;
        keep[1] = true;
        break;
    case OP_FIX:      // d = a - b; b = 2^e d; a = a + d
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) {
            const i64 d = x[0][q] - x[1][q];
            x[0][q] += d;
            x[1][q] = d;
        }
        wv_rot_set<U, F, 2>(x, only(1), slot0, [&](int) -> u64 { return e; }, a.N, l, stage, lane);
        keep[1] = true;
        break;
    case OP_TWOXMY:   // a = 2a - b
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) x[0][q] = 2 * x[0][q] - x[1][q];
        break;
    default:          // OP_IBFLY: t = 2^-e b; a, b = a + t, a - t
        wv_rot_set<U, F, 2>(x, only(1), slot0, [&](int) -> u64 { return e ? N2 - e : 0; }, a.N, l, stage, lane);
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) {
            const i64 s = x[0][q] + x[1][q], d = x[0][q] - x[1][q];
            x[0][q] = s;
            x[1][q] = d;
        }
        keep[1] = true;
        break;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (keep[k]) wv_normalize_store<U, F>(x[k], false, st, slot[k], l, lane);
}

// scaling by 2^-(depth+1) and canonicalisation (mul_fft.c:3256-3260), one wave per coefficient
template <int U, bool F>
__global__ __launch_bounds__(64 * WPB) void k_wscale(u64 *dig, u64 *cb, int *top, int l, u64 N, u64 e, long cnt)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = wv_lane();
    const int wv = wv_id();
    i64 *stage = (i64 *)smem + (size_t)wv * 2 * l;
    const long slot = (long)blockIdx.x * WPB + wv;
    if (slot >= cnt) return;
    Coef st;
    st.dig = dig;
    st.cb = cb;
    st.top = top;
    i64 x[1][2 * U];
    wv_load<U, F>(x[0], st, slot, l, lane);
    wv_rot_set<U, F, 1>(x, [](int) { return true; }, [](int) { return 0; }, [&](int) -> u64 { return e; }, N, l, stage,
                     lane);
    wv_normalize_store<U, F>(x[0], true, st, slot, l, lane);
}
