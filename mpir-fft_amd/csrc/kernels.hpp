// kernels.hpp -- the HIP kernels of the MI355X new_mpn_mul path (gfx950).
//
// Kernel map (DESIGN.md "Kernels"; reference functions in SURVEY 8a):
//   k_pass<U,LOGG,DIR>  2^LOGG coefficients of one column or row in registers,
//                       LOGG radix-2 levels (DIF forward / DIT inverse) with
//                       carry-save digits, one carry resolution at the store.
//                       Covers FFT_split_bits (fused into the first column
//                       pass), FFT_radix2_truncate_twiddle / FFT_radix2_twiddle /
//                       FFT_radix2 / IFFT_radix2 / IFFT_radix2_twiddle
//                       (mul_fft.c:1179, :1397, :786, :1444, :1964) and the MFA
//                       twiddles (README:89; applied at the row pass).
//   k_pairop<U>         the element-wise steps of the truncated inverse
//                       (IFFT_radix2_truncate_twiddle :1733 and
//                       IFFT_radix2_truncate1_twiddle :1604).
//   k_pointwise<U>      new_mpn_mulmod_2expp1 (mul_fft.c:3119 -> MPIR
//                       mpn_mulmod_2expp1): negacyclic 32-bit digit convolution,
//                       one workgroup per product.
//   k_scale<U>          the 2^-(depth+1) scaling + normmod loop (mul_fft.c:3256-3260).
//   k_comb_sum / k_carry_blocks / k_carry_apply
//                       FFT_combine_bits (mul_fft.c:207) as limb-parallel
//                       shifted sums plus a device-wide carry-lookahead.
#pragma once
#include "coeff.hpp"

struct PassArgs {
    u64 *dig[2];
    int *top[2];
    const u64 *src[2];   // non-null: load coefficients straight from the operand (fused split)
    long nsrc[2];
    u64 bits1;
    u64 N;               // bits
    int l;               // limbs
    int lbM, lvl0;       // log2 transform length; first level of this pass
    u64 rho;             // exponent (bits) of the transform's root at level 0
    long sub_stride, pos_stride;
    int nsub, pos_off;
    int zero_from;       // forward: positions >= zero_from are zero inputs
    int need;            // forward: only blocks starting below `need` are live
    int tw_mode;         // 1: pre-multiply by 2^(tw_w*pos*revbin(sub)), 2: post-multiply by its inverse
    u64 tw_w;
    int tw_lbR;
    int canon;           // canonical store (pointwise inputs)
    int ngroups;         // groups per sub-array
    int nbuf;            // LDS staging buffers (1 or 2)
};

// LDS carve: [stage0: 2l i64][stage1: 2l i64 if nbuf == 2][scan scratch]
__device__ __forceinline__ u64 *scan_scratch(unsigned char *smem, int l, int nbuf)
{
    return (u64 *)(smem + (size_t)nbuf * 2 * l * sizeof(i64));
}

template <int U>
struct Rotor {
    const WG &c;
    i64 *st0, *st1;
    int nbuf, l;
    u64 N;
    int rc;
    __device__ Rotor(const WG &c_, i64 *s0, i64 *s1, int nb, int l_, u64 N_)
        : c(c_), st0(s0), st1(s1), nbuf(nb), l(l_), N(N_), rc(0) {}
    // x <- x * 2^e mod p.  e must be workgroup-uniform.
    __device__ __forceinline__ void operator()(i64 (&x)[2 * U], u64 e)
    {
        const Rot r = make_rot(e, N);
        i64 *st = (nbuf > 1 && (rc & 1)) ? st1 : st0;
        ++rc;
        rot_write<U>(c, x, st, l);
        __syncthreads();
        rot_read<U>(c, x, st, r, l);
        if (nbuf == 1) __syncthreads();
    }
    __device__ __forceinline__ void drain() { if (nbuf > 1) __syncthreads(); }
};

template <int U, int LOGG, int DIR>
__global__ __launch_bounds__(1024) void k_pass(PassArgs a)
{
    constexpr int G = 1 << LOGG;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WG c = wg_ctx();
    const int l = a.l;
    i64 *st0 = (i64 *)smem;
    i64 *st1 = st0 + 2 * l;
    u64 *scr = scan_scratch(smem, l, a.nbuf);
    const int op = blockIdx.y;
    u64 *dig = a.dig[op];
    int *top = a.top[op];
    const int sub = (int)(blockIdx.x / a.ngroups);
    const int grp = (int)(blockIdx.x % a.ngroups);
    const int lobits = a.lbM - a.lvl0 - LOGG;
    const int lo = grp & ((1 << lobits) - 1);
    const int hi = grp >> lobits;
    const int bstart = hi << (a.lbM - a.lvl0);
    if (DIR == 0 && bstart >= a.need) return;  // whole block past the truncation point
    const u64 N2 = 2 * a.N;
    const long sbase = (long)sub * a.sub_stride;

    int pos[G];
    long slot[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        pos[i] = bstart | (i << lobits) | lo;
        slot[i] = sbase + (long)(a.pos_off + pos[i]) * a.pos_stride;
    }

    i64 x[G][2 * U];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        if (DIR == 0 && pos[i] >= a.zero_from) zero_coeff<U>(x[i]);
        else if (a.src[op]) load_split<U>(c, x[i], a.src[op], a.nsrc[op], slot[i], a.bits1, l);
        else load_coeff<U>(c, x[i], dig, top, slot[i], l);
    }

    Rotor<U> rot(c, st0, st1, a.nbuf, l, a.N);
    const long rsub = (a.tw_mode) ? revbin_dev(sub, a.tw_lbR) : 0;
    if (a.tw_mode == 1) {
#pragma unroll
        for (int i = 0; i < G; ++i) {
            u64 e = (a.tw_w * (u64)(a.pos_off + pos[i]) * (u64)rsub) % N2;
            if (e) rot(x[i], e);
        }
    }

#pragma unroll
    for (int li = 0; li < LOGG; ++li) {
        const int level = DIR == 0 ? a.lvl0 + li : a.lvl0 + LOGG - 1 - li;
        const int jb = DIR == 0 ? LOGG - 1 - li : li;
        const int h = 1 << (a.lbM - level - 1);
        const u64 unit = (a.rho << level) % N2;
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if ((i >> jb) & 1) continue;
            const int k = i | (1 << jb);
            const u64 e = ((u64)(pos[i] & (h - 1)) * unit) % N2;
            if (DIR == 0) {
#pragma unroll
                for (int q = 0; q < 2 * U; ++q) {
                    const i64 s = x[i][q] + x[k][q], d = x[i][q] - x[k][q];
                    x[i][q] = s;
                    x[k][q] = d;
                }
                if (e) rot(x[k], e);
            } else {
                if (e) rot(x[k], N2 - e);
#pragma unroll
                for (int q = 0; q < 2 * U; ++q) {
                    const i64 s = x[i][q] + x[k][q], d = x[i][q] - x[k][q];
                    x[i][q] = s;
                    x[k][q] = d;
                }
            }
        }
    }

    if (a.tw_mode == 2) {
#pragma unroll
        for (int i = 0; i < G; ++i) {
            u64 e = (a.tw_w * (u64)(a.pos_off + pos[i]) * (u64)rsub) % N2;
            if (e) rot(x[i], N2 - e);
        }
    }
    __syncthreads();

#pragma unroll
    for (int i = 0; i < G; ++i) {
        if (DIR == 0) {
            const int fstart = pos[i] & ~((1 << lobits) - 1);
            if (fstart >= a.need) continue;
        }
        u64 y[U];
        const int tv = wg_normalize<U>(c, x[i], y, l, a.canon != 0, st0, scr);
        store_coeff<U>(c, y, tv, dig, top, slot[i], l);
    }
}

// --------------------------------------------------------------------------
// element-wise steps of the truncated inverse column transform
// --------------------------------------------------------------------------
enum { OP_DOUBLE = 0, OP_HALFADD = 1, OP_FILL = 2, OP_FIX = 3, OP_TWOXMY = 4, OP_IBFLY = 5 };

struct PairArgs {
    u64 *dig;
    int *top;
    u64 N;
    int l;
    int op;
    long NC;      // slot stride between rows
    int ncol;
    int off, h, i0, cnt;
    u64 rho;      // e_i = i * rho (mod 2N)
};

template <int U>
__global__ __launch_bounds__(1024) void k_pairop(PairArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WG c = wg_ctx();
    const int l = a.l;
    i64 *st = (i64 *)smem;
    u64 *scr = scan_scratch(smem, l, 1);
    const int col = (int)(blockIdx.x % a.ncol);
    const int i = a.i0 + (int)(blockIdx.x / a.ncol);
    const long sa = (long)(a.off + i) * a.NC + col;
    const long sb = (long)(a.off + i + a.h) * a.NC + col;
    const u64 N2 = 2 * a.N;
    const u64 e = ((u64)i * a.rho) % N2;
    Rotor<U> rot(c, st, st, 1, l, a.N);
    i64 xa[2 * U], xb[2 * U];
    u64 y[U];
    int tv;
    load_coeff<U>(c, xa, a.dig, a.top, sa, l);
    switch (a.op) {
    case OP_DOUBLE:
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) xa[q] *= 2;
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sa, l);
        break;
    case OP_HALFADD:  // a = (a + b) / 2
        load_coeff<U>(c, xb, a.dig, a.top, sb, l);
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) xa[q] += xb[q];
        rot(xa, N2 - 1);
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sa, l);
        break;
    case OP_FILL:     // b = 2^e a
        if (e) rot(xa, e);
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sb, l);
        break;
    case OP_FIX:      // d = a - b; b = 2^e d; a = a + d
        load_coeff<U>(c, xb, a.dig, a.top, sb, l);
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) {
            const i64 d = xa[q] - xb[q];
            xa[q] += d;
            xb[q] = d;
        }
        if (e) rot(xb, e);
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sa, l);
        tv = wg_normalize<U>(c, xb, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sb, l);
        break;
    case OP_TWOXMY:   // a = 2a - b
        load_coeff<U>(c, xb, a.dig, a.top, sb, l);
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) xa[q] = 2 * xa[q] - xb[q];
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sa, l);
        break;
    default:          // OP_IBFLY: t = 2^-e b; a, b = a + t, a - t
        load_coeff<U>(c, xb, a.dig, a.top, sb, l);
        if (e) rot(xb, N2 - e);
#pragma unroll
        for (int q = 0; q < 2 * U; ++q) {
            const i64 s = xa[q] + xb[q], d = xa[q] - xb[q];
            xa[q] = s;
            xb[q] = d;
        }
        tv = wg_normalize<U>(c, xa, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sa, l);
        tv = wg_normalize<U>(c, xb, y, l, false, st, scr);
        store_coeff<U>(c, y, tv, a.dig, a.top, sb, l);
        break;
    }
}

// --------------------------------------------------------------------------
// scaling by 2^-(depth+1) and canonicalisation (mul_fft.c:3256-3260)
// --------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(1024) void k_scale(u64 *dig, int *top, int l, u64 N, u64 e)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WG c = wg_ctx();
    i64 *st = (i64 *)smem;
    u64 *scr = scan_scratch(smem, l, 1);
    const long slot = blockIdx.x;
    i64 x[2 * U];
    u64 y[U];
    load_coeff<U>(c, x, dig, top, slot, l);
    Rotor<U> rot(c, st, st, 1, l, N);
    if (e) rot(x, e);
    const int tv = wg_normalize<U>(c, x, y, l, true, st, scr);
    store_coeff<U>(c, y, tv, dig, top, slot, l);
}

// --------------------------------------------------------------------------
// pointwise products mod 2^N + 1 (one workgroup per slot), in place into A.
//   a b == sum_k Q_k X^k + S - a  (mod X^L + 1, X = 2^32), with
//   Q_k = sum_i a_i B'_{k-i+L},  B'_m = ~b_m (m < L), b_{m-L} (m >= L),
//   S = sum_i a_i.  Every column has exactly L unsigned terms (no divergence);
//   the complement trick turns the negacyclic wrap into the "- a + S" fix-up.
// LDS: A[L] u32, B'[2L] u32 (then reused as normalisation scratch).
// --------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(1024) void k_pointwise(u64 *digA, int *topA, const u64 *digB, const int *topB,
                                                    int l, u64 N)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WG c = wg_ctx();
    const int L = 2 * l;
    u32 *As = (u32 *)smem;
    u32 *Bs = As + L;
    u64 *scr = (u64 *)(smem + (size_t)3 * L * sizeof(u32));
    u64 *ssum = scr + 3 * U * 16 + 4;
    const long slot = blockIdx.x;
    const int ta = topA[slot], tb = topB[slot];  // canonical inputs: tops in {0, 1}
    const u64 *pa = digA + (size_t)slot * l;
    const u64 *pb = digB + (size_t)slot * l;
    u64 asum = 0;
    if (c.t == 0) *ssum = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int m = u * c.nt + c.t;
        if (m < l) {
            const u64 va = pa[m], vb = pb[m];
            As[2 * m] = (u32)va;
            As[2 * m + 1] = (u32)(va >> 32);
            Bs[L + 2 * m] = (u32)vb;
            Bs[L + 2 * m + 1] = (u32)(vb >> 32);
            Bs[2 * m] = ~(u32)vb;
            Bs[2 * m + 1] = ~(u32)(vb >> 32);
            asum += (va & MPF_M32) + (va >> 32);
        }
    }
    __syncthreads();
    i64 d[2 * U];
    if (ta | tb) {
        // 2^N == -1: the product is -b, -a or 1 (MPIR's c flags, mul_fft.c:3250)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            d[2 * u] = d[2 * u + 1] = 0;
            if (m < l) {
                if (ta && tb) {
                    d[2 * u] = (m == 0) ? 1 : 0;
                } else {
                    const u32 *o = ta ? (Bs + L) : As;
                    d[2 * u] = -(i64)o[2 * m];
                    d[2 * u + 1] = -(i64)o[2 * m + 1];
                }
            }
        }
        __syncthreads();
    } else {
        for (int off = 32; off > 0; off >>= 1) asum += __shfl_xor(asum, off);
        if (c.lane == 0) atomicAdd((unsigned long long *)ssum, (unsigned long long)asum);
        u64 r1[U];
        i64 q0[2 * U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            q0[2 * u] = q0[2 * u + 1] = 0;
            r1[u] = 0;
            if (m < l) {
                const int k0 = 2 * m;
                u64 acc0 = 0, acc1 = 0;
                u32 h0 = 0, h1 = 0;
                const u32 *bp = Bs + k0 + L;
                for (int i = 0; i < L; ++i) {
                    const u64 av = As[i];
                    const u64 p0 = av * bp[-i];
                    const u64 p1 = av * bp[1 - i];
                    acc0 += p0;
                    h0 += (acc0 < p0);
                    acc1 += p1;
                    h1 += (acc1 < p1);
                }
                // Q_k = q0_k + r_k X with r_k = Q_k >> 32 (< 2^45)
                const u64 rk0 = (acc0 >> 32) | ((u64)h0 << 32);
                const u64 rk1 = (acc1 >> 32) | ((u64)h1 << 32);
                q0[2 * u] = (i64)(acc0 & MPF_M32) - (i64)As[k0];
                q0[2 * u + 1] = (i64)(acc1 & MPF_M32) - (i64)As[k0 + 1] + (i64)rk0;
                r1[u] = rk1;
            }
        }
        __syncthreads();
        i64 *sh = (i64 *)smem;  // As/Bs are dead now
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            if (m < l) sh[m] = (i64)r1[u];
        }
        __syncthreads();
        const i64 S = (i64)*ssum;
        const i64 rl = sh[l - 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int m = u * c.nt + c.t;
            d[2 * u] = q0[2 * u];
            d[2 * u + 1] = q0[2 * u + 1];
            if (m < l) d[2 * u] += m ? sh[m - 1] : (S - rl);  // X^L == -1 wraps r_{L-1}
        }
        __syncthreads();
    }
    u64 y[U];
    const int tv = wg_normalize<U>(c, d, y, l, true, (i64 *)smem, scr);
    store_coeff<U>(c, y, tv, digA, topA, slot, l);
}

// --------------------------------------------------------------------------
// combine: r = sum_{k < len} c_k 2^(k bits1), c_k < 2^N canonical.
// k_comb_sum: per output limb m, the 128-bit sum of the (at most a few)
// coefficient windows covering bits [64m, 64m + 64); lo -> lo64[m], hi -> hi32[m].
// The carry chain r = lo + (hi << 64) is then resolved by a device-wide
// carry-lookahead (k_carry_blocks -> k_carry_scan -> k_carry_apply).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_comb_sum(const u64 *dig, int l, u64 N, u64 bits1, long len, long total,
                                                  u64 *lo64, u32 *hi32)
{
    const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= total) return;
    const u64 P = (u64)m * 64;
    long klo = (P >= N) ? (long)((P - N) / bits1) : 0;
    long khi = (long)((P + 63) / bits1);
    if (khi > len - 1) khi = len - 1;
    u64 slo = 0;
    u32 shi = 0;
    for (long k = klo; k <= khi; ++k) {
        const u64 st = (u64)k * bits1;
        const u64 *cp = dig + (size_t)k * l;
        u64 v;
        if (st > P) {
            v = cp[0] << (st - P);
        } else {
            const u64 o = P - st;
            const long q = (long)(o >> 6);
            const int s = (int)(o & 63);
            const u64 w0 = (q < l) ? cp[q] : 0;
            const u64 w1 = (s && q + 1 < l) ? cp[q + 1] : 0;
            v = s ? (w0 >> s) | (w1 << (64 - s)) : w0;
        }
        u64 t;
        shi += add_ovf(slo, v, &t);
        slo = t;
    }
    lo64[m] = slo;
    hi32[m] = shi;
}

// limb m of the final sum is e_m = lo64[m] + hi32[m-1]: value v, generate g, propagate p
__device__ __forceinline__ void carry_limb(const u64 *lo64, const u32 *hi32, long m, u64 *v, bool *g, bool *p)
{
    const u64 add = m ? hi32[m - 1] : 0;
    *g = add_ovf(lo64[m], add, v);
    *p = (*v == MPF_MAXL);
}

#define CARRY_V 8  // limbs per thread in the carry kernels (256 threads -> 2048 limbs per block)

// per-thread (generate, propagate) over its CARRY_V contiguous limbs
__device__ __forceinline__ void carry_thread(const u64 *lo64, const u32 *hi32, long m0, long total, bool *G, bool *P)
{
    bool g = false, p = true;
    for (int k = 0; k < CARRY_V; ++k) {
        long m = m0 + k;
        if (m >= total) break;
        u64 v;
        bool gk, pk;
        carry_limb(lo64, hi32, m, &v, &gk, &pk);
        g = gk || (pk && g);
        p = p && pk;
    }
    *G = g;
    *P = p;
}

__global__ __launch_bounds__(256) void k_carry_blocks(const u64 *lo64, const u32 *hi32, long total, u8 *blkG, u8 *blkP)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long m0 = ((long)blockIdx.x * blockDim.x + c.t) * CARRY_V;
    bool G, P;
    carry_thread(lo64, hi32, m0, total, &G, &P);
    u32 co;
    wg_scan<1>(c, G, P, 0, &co, scr);
    // block summary: generate = carry out with cin 0; propagate = every thread propagates
    const u64 allp = __ballot(P);
    __shared__ int pall;
    if (c.t == 0) pall = 1;
    __syncthreads();
    if (c.lane == 0 && allp != ~0ull) pall = 0;
    __syncthreads();
    if (c.t == 0) {
        blkG[blockIdx.x] = (u8)co;
        blkP[blockIdx.x] = (u8)(pall && !co);
    }
}

// single workgroup: carry into every block
__global__ __launch_bounds__(1024) void k_carry_scan(const u8 *blkG, const u8 *blkP, long nblk, u8 *blkC)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long per = (nblk + c.nt - 1) / c.nt;
    const long b0 = (long)c.t * per;
    bool g = false, p = true;
    for (long b = b0; b < b0 + per && b < nblk; ++b) {
        g = blkG[b] || (blkP[b] && g);
        p = p && blkP[b];
    }
    u32 co;
    u32 ci = wg_scan<1>(c, g, p, 0, &co, scr);
    bool run = ci & 1;
    for (long b = b0; b < b0 + per && b < nblk; ++b) {
        blkC[b] = (u8)run;
        run = blkG[b] || (blkP[b] && run);
    }
}

__global__ __launch_bounds__(256) void k_carry_apply(const u64 *lo64, const u32 *hi32, long total, const u8 *blkC,
                                                     u64 *r)
{
    __shared__ u64 scr[64];
    const WG c = wg_ctx();
    const long m0 = ((long)blockIdx.x * blockDim.x + c.t) * CARRY_V;
    bool G, P;
    carry_thread(lo64, hi32, m0, total, &G, &P);
    u32 co;
    const u32 ci = wg_scan<1>(c, G, P, blkC[blockIdx.x], &co, scr);
    bool run = ci & 1;
    for (int k = 0; k < CARRY_V; ++k) {
        long m = m0 + k;
        if (m >= total) break;
        u64 v;
        bool gk, pk;
        carry_limb(lo64, hi32, m, &v, &gk, &pk);
        r[m] = v + (run ? 1 : 0);
        run = gk || (pk && run);
    }
}
