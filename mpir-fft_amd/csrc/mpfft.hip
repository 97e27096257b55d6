// mpfft.hip -- host orchestration and C ABI of the MI355X-native new_mpn_mul.
//
// The drop-in boundary is new_mpn_mul(r1, i1, n1, i2, n2, depth, w)
// (/root/reference/mul_fft.c:3190-3191); see include/mpfft.h.  Everything below
// the boundary is a re-design for gfx950:
//
//   1. forward column pass(es): split fused into the first pass; truncated DIF of
//      length NR on every column, both operands in one launch        (a2-a12)
//   2. forward row pass(es): MFA twiddle fused into the load, DIF of length NC
//      over the T/NC live rows, canonical store                       (a3, a7)
//   3. pointwise mulmod 2^N+1 over the T live slots                   (a20)
//   4. inverse row pass(es), MFA un-twiddle fused into the store      (a13, a15)
//   5. truncated inverse column transform (van der Hoeven), driven as a host
//      recursion of block IFFT passes and element-wise pair steps     (a13, a14)
//   6. scale by 2^-(depth+1) + canonicalise                           (a21)
//   7. combine: limb-parallel shifted sums + device-wide carry scan   (a22)
//
// Slot layout: operand X lives in slots 0..2n-1 (row-major, NC columns).  After
// stage 2, slot p*NC + q holds X_{revbin(p) + NR*revbin(q)} (the reference's
// slot map, mul_fft.c:2357, up to its two revbin permutations, which we never
// perform because the inverse undoes them).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <mutex>
#include <vector>

#include "kernels.hpp"
#include "combine.hpp"
#include "fold.hpp"
#include "wdispatch.hpp"
#include "bdispatch.hpp"
#include "pdispatch.hpp"
#include "rdispatch.hpp"
#include "../../include/mpfft.h"

// ---------------------------------------------------------------------------
// parameters (mul_fft.c:3193-3203)
// ---------------------------------------------------------------------------
// Tuning / ablation / stamp knobs exist only in a diagnostic build (make DIAG=1 defines
// MPFFT_DIAG); the shipped library never reads them, so no environment can make it skip
// work or run an untested kernel family.
static const char *diag_env(const char *name)
{
#ifdef MPFFT_DIAG
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// wave kernels for coefficients of l limbs: U = ceil(l / 64) limbs per lane, full rows when l == 64 U
static WvFns wv_fns(int U, bool full)
{
    switch (U) {
    case 1: return full ? wv_fns_u1_1() : wv_fns_u1_0();
    case 2: return full ? wv_fns_u2_1() : wv_fns_u2_0();
    case 3: return full ? wv_fns_u3_1() : wv_fns_u3_0();
    default: return full ? wv_fns_u4_1() : wv_fns_u4_0();
    }
}

struct Plan {
    long n1, n2;
    int depth;
    long w;
    long n, l;
    u64 N, bits1;
    long NC, NR;
    int lbC, lbR;
    long j1, j2, trunc, Tr, len, total;
    int U, tpb, maxlogg;
    int maxlogg_c;      // column passes (forward and inverse); maxlogg: row passes
    int maxlogg_i;      // inverse (DIT) k_rpass passes, rows and columns (0: as above)
    int bp_lg;          // most levels k_bpass fits in LDS (big): a pass k_rpass declines is capped to it
    bool wave;          // wave-owned coefficient kernels (wkernels.hpp), l <= 512
    int wU;             // their limbs per lane
    bool wfull;         // l == 64 wU
    bool fuse_scale;    // scaling fused into the last inverse column pass (no truncation)
    bool lds;           // LDS-resident radix-2^5 passes (lkernels.hpp)
    bool big;           // LDS-resident passes for 512 <= l <= 4096 (bkernels.hpp)
    bool rpass;         // register-resident passes (rkernels.hpp) where they apply, l = 1024, 2048, 4096
    bool sqrt2;         // new_mpn_mul6 plan: 4n slots, bits1 = (N - depth - 1)/2, Tr up to 2 NR
    size_t slots;       // allocated slots per operand
    // off_flags: k_combine1's look-back flags + ticket counter, cleared by the first forward
    // column pass
    // (Exec::zflags) -- no stage between that pass and the combine may use this region
    size_t off_digA, off_topA, off_cbA, off_digB, off_topB, off_cbB, off_flags, bytes;
    bool has_c;         // a third coefficient array C: the fused pointwise (k_pwss PAIR) writes there
    int fold;           // f4 (fold.hpp): scaling in the last inverse row pass, reduced-form combine with
                        // KM = fold coefficients per wave (0: k_rscale + k_combine1)
    bool ltw;           // fold plans: the inverse MFA twiddle and the scaling ride in the first pass of
                        // each column block of the truncated inverse (k_rpass DIT mode bit 3) instead
                        // of the rows' last pass (every block's rotation a whole number of limb pairs)
    size_t off_meta;    // k_cmeta's per-coefficient A_k, B_k (fold plans)
    int fuse_rows;      // row DIF levels that run inside the pointwise: 1 (slot pairs), 2 (slot quads), 0
    size_t off_digC, off_topC, off_cbC;
};

static int ilog2(long v) { int d = 0; while ((1L << d) < v) ++d; return d; }

// pointwise kernel family.  MPFFT_POINTWISE is the one runtime selector the shipped library
// reads (every choice is an exact product; the parity tests A/B them): auto (default),
// pwss = the nested negacyclic k_pwss (l = 1024, 2048, 4096), mfma = int8-MFMA k_pwm2
// (l % 256 == 0), mfma1 = k_pwm (l % 128 == 0), valu = k_pw.
enum { PW_AUTO = 0, PW_PWSS, PW_MFMA, PW_MFMA1, PW_VALU };
static int pw_kind()
{
    const char *e = getenv("MPFFT_POINTWISE");
    if (!e) return PW_AUTO;
    if (!strcmp(e, "pwss")) return PW_PWSS;
    if (!strcmp(e, "mfma")) return PW_MFMA;
    if (!strcmp(e, "mfma1")) return PW_MFMA1;
    if (!strcmp(e, "valu")) return PW_VALU;
    return PW_AUTO;
}

// nested negacyclic pointwise (pkernels.hpp) for big coefficients: log2 of its piece count
// (0: another kernel).  Default from l = 2048 on; at l = 1024 the int8-MFMA schoolbook wins.
static int pwss_lk_of(long l)
{
    const int k = pw_kind();
    if (k != PW_AUTO && k != PW_PWSS) return 0;
    switch (l) {
    case 1024: return k != PW_AUTO ? 8 : 0;
    case 2048: return 8;
    case 4096: return 9;   // K = 1024 (M = 16, 1024 threads, 4 waves/SIMD) measured slower: C4 63.3 vs 45.3 ms
    }
    return 0;
}

// the fused-pair k_pwss instance (last row DIF level on load, product to C) exists for l;
// fuse 2: the fused-quad instance (the last two levels)
static bool pw_pair_kernel(long l, int fuse = 1)
{
    const int lk = pwss_lk_of(l);
    return lk && pw_get(pw_inner_limbs(l, lk), lk, fuse) != nullptr;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// sqrt2: the new_mpn_mul6 front end (mul_fft.c:3573-3603): a length-4n convolution with
// bits1 = (N - (depth + 1))/2 (:3578) and the same trunc rule (:3603)
// lbc >= 0: NC = 2^lbc instead of the reference's split; fwd4: four-level forward k_rpass passes
static int make_plan_split(Plan *p, long n1, long n2, unsigned long depth, unsigned long w, bool sqrt2, int lbc,
                           bool fwd4 = false)
{
    memset(p, 0, sizeof(*p));
    p->sqrt2 = sqrt2;
    if (n1 < 1 || n2 < 1) return MPFFT_EINVAL;
    if (depth < 2 || depth > 30 || w < 1 || w > 4096) return MPFFT_EINVAL;
    p->n1 = n1;
    p->n2 = n2;
    p->depth = (int)depth;
    p->w = (long)w;
    p->n = 1L << depth;
    if (((u64)p->n * w) % 64) return MPFFT_EINVAL;          // N must be a whole number of limbs
    p->N = (u64)p->n * w;
    p->l = (long)(p->N / 64);
    if (p->N <= depth) return MPFFT_EINVAL;
    if (sqrt2 && p->N <= depth + 1) return MPFFT_EINVAL;
    p->bits1 = (p->N - depth - (sqrt2 ? 1 : 0)) / 2;
    if (p->bits1 < 1) return MPFFT_EINVAL;
    p->NC = 1L << (lbc >= 0 ? lbc : (int)depth / 2);   // the reference's split (mul_fft.c:3195) unless make_plan picks another
    p->NR = 2 * p->n / p->NC;
    p->lbC = ilog2(p->NC);
    p->lbR = ilog2(p->NR);
    p->j1 = (long)((64 * (u64)n1 - 1) / p->bits1 + 1);
    p->j2 = (long)((64 * (u64)n2 - 1) / p->bits1 + 1);
    p->len = p->j1 + p->j2 - 1;
    if (p->len > (sqrt2 ? 4 : 2) * p->n) return MPFFT_ETOOBIG;   // product does not fit the convolution
    p->trunc = ((p->j1 + p->j2 - 2 + 2 * p->NC) / (2 * p->NC)) * 2 * p->NC;
    p->Tr = p->trunc / p->NC;
    p->total = n1 + n2;
    if (p->l > 4096) return MPFFT_EUNSUPPORTED;              // pointwise LDS budget (24 l bytes)
    // threads per coefficient and limbs per thread: U == 1 kernels are built for
    // <= 256 threads (MPF_LB), U == 2 / 4 for <= 1024
    const int Up = p->l <= 256 ? 1 : p->l <= 2048 ? 2 : 4;
    long tpb = 64;
    while (tpb * Up < p->l) tpb *= 2;
    p->tpb = (int)tpb;
    p->U = Up;
    p->maxlogg = Up == 1 ? 4 : Up == 2 ? 2 : 1;   // G*U <= 8 keeps U >= 2 passes spill-free
    {
        const char *e = diag_env("MPFFT_WAVE");
        p->wave = p->l <= 256 && !(e && !strcmp(e, "0"));
    }
    if (p->wave) {
        p->wU = (int)((p->l + 63) / 64);
        p->wfull = p->l == 64L * p->wU;
        p->maxlogg = wv_fns(p->wU, p->wfull).maxlogg;
        const char *e = diag_env("MPFFT_WLOGG");
        if (e && atoi(e) >= 1 && atoi(e) <= p->maxlogg) p->maxlogg = atoi(e);
        p->fuse_scale = p->Tr == p->NR && !sqrt2;
        const char *el = diag_env("MPFFT_LDS");
        p->lds = !(el && !strcmp(el, "0"));
        if (p->lds) {
            p->maxlogg = LP_MAXLOGG;
            if (e && atoi(e) >= 1 && atoi(e) <= LP_MAXLOGG) p->maxlogg = atoi(e);
        }
    }
    {
        const char *e = diag_env("MPFFT_BIG");
        const long rows = p->l / 64;
        p->big = !p->wave && p->l >= 512 && p->l % 64 == 0 && !(rows & (rows - 1)) && !(e && !strcmp(e, "0"));
    }
    if (p->big) {   // as many levels per pass as coefficients fit in LDS (G <= 16)
        int lg = 1;
        while (lg < BP_MAXLOGG && bp_lds_need(p->l, 2 << lg) <= BP_LDS_MAX) ++lg;
        p->maxlogg = lg;
        p->bp_lg = lg;
        // columns: two 74 KB groups per CU beat one 147 KB group at l = 2048 (C3 sweep,
        // profiles/r02/sweep_blogg.txt: columns 5.97 ms vs 6.53 ms; rows 4.71 vs 4.44)
        p->maxlogg_c = lg >= 3 ? lg - 1 : lg;
        const char *e = diag_env("MPFFT_BLOGG");
        if (e && atoi(e) >= 1 && atoi(e) <= lg) p->maxlogg = p->maxlogg_c = atoi(e);
        const char *er = diag_env("MPFFT_RPASS");
        p->rpass = rp_maxlogg((int)p->l) > 0 && !(er && !strcmp(er, "0")) && !diag_env("MPFFT_BP_STAMPS");
        if (p->rpass && !e) {   // same levels per pass for columns and rows (two groups per CU either way)
            int rl = fwd4 ? rp_maxlogg_fwd4((int)p->l) : rp_maxlogg((int)p->l);   // register-resident: not bound by k_bpass's LDS fit
            const char *ec = diag_env("MPFFT_RPLOGG");   // diagnostics: fewer levels per pass (A/B)
            if (ec && atoi(ec) >= 1 && atoi(ec) < rl) rl = atoi(ec);
            p->maxlogg = p->maxlogg_c = rl;
            int ri = rp_maxlogg_dit((int)p->l);
            const char *ei = diag_env("MPFFT_RPLOGG_INV");
            if (ei && atoi(ei) >= 1 && atoi(ei) < ri) ri = atoi(ei);
            if (ec && rl < ri) ri = rl;
            p->maxlogg_i = ri;
        }
    }
    p->slots = (size_t)(sqrt2 ? 4 : 2) * p->n;
    size_t o = 0;
    const size_t dig = p->slots * p->l * 8, top = align_up(p->slots * 4, 256);
    const size_t cbb = align_up(p->slots * cb_words((int)p->l) * 8, 256);
    p->off_digA = o; o += dig;
    p->off_topA = o; o += top;
    p->off_cbA = o; o += cbb;
    p->off_digB = o; o += dig;
    p->off_topB = o; o += top;
    p->off_cbB = o; o += cbb;
    // C: output of the fused last-row-level pointwise (single-GPU new_mpn_mul, Exec::row_fused)
    // (only where it saves a row pass: fewer passes for lbC - 1 levels than for lbC)
    {
        // the last two levels where that saves a pass and one does not (C4: 8 row levels at <= 3
        // per pass are 3 + 3 + 2, 6 are 3 + 3); the quad form needs the plain MFA row root (not
        // the sqrt2 front end's)
        const int ml = p->maxlogg > 0 ? p->maxlogg : 1;
        auto np = [&](int L) { return (L + ml - 1) / ml; };
        const bool f1 = p->lbC >= 2 && np(p->lbC - 1) < np(p->lbC) && pw_pair_kernel(p->l);
        static const bool no2 = diag_env("MPFFT_NO_FUSE2") != nullptr;   // diagnostics: A/B
        const int lk = pwss_lk_of(p->l);   // quad inputs are 4x the pieces: 2 more bits of headroom (pdispatch.hpp)
        const bool room = lk && 64 * pw_inner_limbs(p->l, lk) >= 2 * ((64 * p->l) >> lk) + lk + 6;
        // ... or where it turns four-level row passes into three-level ones (8 row levels: 4 + 4 ->
        // fused 2 + 3 + 3 -- three-level passes run two workgroups per CU; C3 8.64 -> 8.55 ms,
        // profiles/r04/quad_fuse_ab.txt)
        const bool saves2 = np(p->lbC - 2) < np(p->lbC - 1) && np(p->lbC - 2) < np(p->lbC);
        const bool to3 = ml == 4 && p->lbC - 2 == 6;
        const bool f2 = !sqrt2 && !no2 && room && p->lbC >= 3 && (saves2 || to3) && pw_pair_kernel(p->l, 2);
        static const bool force2 = diag_env("MPFFT_FORCE_FUSE2") != nullptr;   // diagnostics: A/B
        const bool f2f = force2 && !sqrt2 && room && p->lbC >= 3 && pw_pair_kernel(p->l, 2);
        p->fuse_rows = (f2 || f2f) ? 2 : f1 ? 1 : 0;
        p->has_c = p->fuse_rows > 0;
    }
    if (p->has_c) {
        p->off_digC = o; o += dig;
        p->off_topC = o; o += top;
        p->off_cbC = o; o += cbb;
    }
    p->off_flags = o; o += align_up((size_t)(p->total / 256 + 8) * 4, 256);   // k_combine1 blocks at V = 1
    // f4 fold (fold.hpp) on the truncated register-pass plans: KM coefficients reach a wave's 512
    // product limbs (windows shifted by up to one bit); MPFFT_FOLD=0 (diagnostics): k_rscale + k_combine1
    {
        static const bool no_fold = [] { const char *e = diag_env("MPFFT_FOLD"); return e && !strcmp(e, "0"); }();
        const int km = (int)((p->N + 1 + 32767) / p->bits1 + 1);
        p->fold = (p->rpass && !sqrt2 && p->Tr < p->NR && p->bits1 > 512 && km <= 4 && !no_fold) ? (km <= 3 ? 3 : 4) : 0;
        static const bool no_ltw = [] { const char *e = diag_env("MPFFT_LTW"); return e && !strcmp(e, "0"); }();
        // where it measured faster: l <= 2048 (C3 inverse rows + columns 1.714 -> 1.679 ms); at
        // l = 4096 the rotated loads in the three-level column passes cost more than the rows save
        // (C4 15.54 -> 15.84 ms), profiles/r06/ltw_ab.txt
        p->ltw = p->fold && ((u64)p->w * (u64)p->NC) % 128 == 0 && p->l <= 2048 && !no_ltw;
    }
    p->off_meta = o; o += align_up((size_t)p->slots * 4, 256);
    p->bytes = o;
    return MPFFT_OK;
}

// rows of the truncated inverse column transform whose top-level doubling Exec::itft leaves to
// the scaling (defer_double): IFFT_radix2_truncate's t <= h branch doubles outputs [0, t), the
// t > h branch [t - h, h) (mul_fft.c:1733-1790)
static void plan_dbl(const Plan &P, long *lo, long *hi)
{
    const long t = P.Tr, h = P.NR / 2;
    *lo = *hi = 0;
    if (t == P.NR) return;
    if (t <= h) *hi = t;
    else {
        *lo = t - h;
        *hi = h;
    }
}

// The matrix split of the MFA is internal (no internal ABI): the reference takes
// NC = 2^floor(depth/2) columns (mul_fft.c:3195).  At l = 2048 with truncation case b
// (trunc > half the convolution), and since round 6 in case a at depth 13-15 as well (below),
// twice the columns with four-level forward passes is faster:
// C3 (depth 15) 256 x 256 runs its 8 column levels in 4 + 4 where 128 x 512 needs 3 + 3 + 3,
// 8.64 vs 8.81 ms; in case a the reference split's column transform skips its empty upper
// half and wins (C2: 6.69 vs 6.99 ms); at l = 4096 (C4) 512 x 512 with three-level passes
// measured slower (97.1 vs 96.2 ms).  profiles/r04/mfa_split_ab.txt.  Both splits give the
// same exact product.
static int make_plan(Plan *p, long n1, long n2, unsigned long depth, unsigned long w, bool sqrt2 = false)
{
    int rc = make_plan_split(p, n1, n2, depth, w, sqrt2, -1);
    // diagnostics (A/B): MPFFT_SPLIT=ref / alt forces a split
    static const char *force = diag_env("MPFFT_SPLIT");
    // l = 4096, truncation case b: twice the reference's columns since the live-group launches (C4 74.1-74.3
    // -> 72.2 ms, profiles/r06/c4_split_ab.txt; round 4, before them, measured it slower); case a unmeasured
    if (!rc && !sqrt2 && p->rpass && p->l == 4096 && !(force && !strcmp(force, "ref"))
        && (2 * p->Tr > p->NR || (force && !strcmp(force, "alt4")))) {
        Plan q;
        if (make_plan_split(&q, n1, n2, depth, w, sqrt2, (int)depth / 2 + 1) == MPFFT_OK && q.rpass) *p = q;
        return rc;
    }
    if (rc || sqrt2 || !p->rpass || p->l != 2048 || (force && !strcmp(force, "ref"))) return rc;
    // case a (2 Tr <= NR) too at depth 13-15 since the live-group launches (C2 6.09 -> 5.95 ms, -2.2 to
    // -4.8 % over truncation ratios 0.40-0.48 at depth 13-15, +0.3-0.5 % at depth 16:
    // profiles/r06/split_resweep.txt); smaller depths were not re-measured and keep the rule
    const bool casea = 2 * p->Tr <= p->NR;
    if (!(force && !strcmp(force, "alt")) && casea && (depth < 13 || depth > 15)) return rc;
    Plan q;
    if (make_plan_split(&q, n1, n2, depth, w, sqrt2, (int)depth / 2 + 1, true) == MPFFT_OK && q.rpass
        && (!casea || (force && !strcmp(force, "alt")) || q.trunc <= p->trunc + p->trunc / 64))   // case a: at most 1/64 more truncated length
        *p = q;
    return MPFFT_OK;
}

// ---------------------------------------------------------------------------
// kernel dispatch
// ---------------------------------------------------------------------------
typedef void (*pass_fn)(PassArgs);

template <int U>
static pass_fn pick_pass(int logg, int dir)
{
    constexpr int ML = U == 1 ? 4 : U == 2 ? 2 : 1;
    if (dir == 0) {
        switch (logg) {
        case 1: return k_pass<U, 1, 0>;
        case 2: if (ML >= 2) return k_pass<U, (ML >= 2 ? 2 : 1), 0>; break;
        case 3: if (ML >= 3) return k_pass<U, (ML >= 3 ? 3 : 1), 0>; break;
        case 4: if (ML >= 4) return k_pass<U, (ML >= 4 ? 4 : 1), 0>; break;
        }
    } else {
        switch (logg) {
        case 1: return k_pass<U, 1, 1>;
        case 2: if (ML >= 2) return k_pass<U, (ML >= 2 ? 2 : 1), 1>; break;
        case 3: if (ML >= 3) return k_pass<U, (ML >= 3 ? 3 : 1), 1>; break;
        case 4: if (ML >= 4) return k_pass<U, (ML >= 4 ? 4 : 1), 1>; break;
        }
    }
    return nullptr;
}

static size_t wpass_lds(int U, int G, int l) { return (size_t)WPB * wv_stage_slots(G, U) * 16 * (size_t)l; }

static pass_fn get_pass(int U, int logg, int dir)
{
    switch (U) {
    case 1: return pick_pass<1>(logg, dir);
    case 2: return pick_pass<2>(logg, dir);
    case 4: return pick_pass<4>(logg, dir);
    }
    return nullptr;
}

// dynamic LDS above 64 KiB must be opted into per kernel (gfx950 has 160 KiB per CU)
static void allow_lds(const void *f, size_t bytes)
{
    if (bytes > 64 * 1024) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { last_hip_error = e_; return MPFFT_EHIP; } } while (0)
static thread_local hipError_t last_hip_error = hipSuccess;
void mpfft_note_hip_error(hipError_t e) { last_hip_error = e; }   // multi.hip's failures

// multi.hip: the device list mpfft_set_devices / MPFFT_DEVICES picks for this product (0: none)
int mpfft_multi_policy(long n1, long n2, unsigned long depth, unsigned long w, std::vector<int> &devs);

// Where one rank's data lives.  The column layout (slot = pos * ccount + c - c0)
// feeds the column passes; the row layout (rows r0 .. r0 + rcount of `nblk` column
// blocks of ccb columns: slot = (c / ccb) * rcount * ccb + (p - r0) * ccb + c % ccb)
// feeds the row passes and the pointwise products.  On one GPU both are the same
// natural slot-major array (c0 = r0 = 0, ccount = ccb = NC, rcount = T/NC).
struct View {
    u64 *dig[2];
    u64 *cb[2];
    int *top[2];
};

struct Exec {
    const Plan &P;
    hipStream_t s;
    int nw;
    View col, row;
    View cview = {};         // the C arrays (single layout, index 0), when the plan has them
    int c0, ccount, r0, rcount, ccb, cbb;
    long cbs;
    long src_chunk = 0;      // operands are column slices (mpfft_shard.src_chunk), 0 = whole operands
    u32 *zflags = nullptr;   // non-null: the first forward column pass clears the combine's look-back flags
    long zflags_n = 0;       // (u32 words), so combine_single needs no separate fill launch
    int in_rows = 0;         // non-zero: inputs live in column rows [0, in_rows) (default: the trunc rows)
    bool defer_double = false;   // itft's top-level doubling is left to scale() (rows [dbl_lo, dbl_hi): 2^-depth)
    bool fold = false;           // f4 (P.fold): 2^-(depth+1) in the last inverse row pass, no scale(), combine_fold()
    bool fuse_row_last = false;  // the row DIF's last level runs inside the pointwise (k_pwss PAIR)
    // forward columns: only output rows [own_lo, own_hi) are wanted (own_hi > 0).  After the
    // first column pass a DIF splits into independent subtrees of positions; the later passes
    // skip the subtrees outside the rows (MPFFT_SHARD_FWD_COLUMNS_OWN: a rank of the replicated
    // forward columns keeps only its own rows of each column block)
    int own_lo = 0, own_hi = 0;
    // forward k_rpass passes hand their pending exponents on to the next pass of the same
    // transform (fwd_columns / fwd_rows).  Every stage still ends exact -- a transform's last
    // level leaves no pending exponent (its pass skips the closing round) -- so the stage API
    // and the sharded path run the same passes.
    bool carry_pend = !diag_env("MPFFT_NO_CARRY");
    // which hand-overs: 1 column -> column, 4 row -> row.  The receiving pass applies the
    // owed exponents (whole limb pairs) by a rotated load -- addresses and a negation, no LDS
    // round -- so its first level stays in registers and the skipped closing round is saved
    // outright.  (Round 3, when the first level took the exponents through LDS instead, the
    // hand-over paid only row -> row and column -> column at l = 4096: profiles/r03/carry_ab.txt.)
    int carry_mask() const
    {
        static const int m = [] { const char *e = diag_env("MPFFT_CARRY_MASK"); return e ? atoi(e) : -1; }();
        return m >= 0 ? m : 5;
    }
    struct Fill { long lo = 0, off = 0; u64 rho = 0; bool done = false; } fill;   // itft's FILL, see ifft_block
    long dbl_lo = 0, dbl_hi = 0;

    Exec(const Plan &p, hipStream_t st) : P(p), s(st) { nw = P.tpb / 64; }

    // levels in the next pass when `rem` remain: the fewest passes of <= maxlogg
    // levels, balanced (C1 column inverse: 4 + 3 beats 5 + 2 by ~5 us)
    int split(int rem, bool col = false, bool inv = false) const
    {
        const int ml = inv && P.maxlogg_i ? P.maxlogg_i : col && P.maxlogg_c ? P.maxlogg_c : P.maxlogg;
        const int np = (rem + ml - 1) / ml;
        return (rem + np - 1) / np;
    }

    // k_combine1 block size: 256 comb_v() limbs (MPFFT_CB_V = 1, 2, 4, 8)
    static int comb_v()
    {
        // C3 sweep (profiles/r02/combine_cbv.txt): V = 1: 1.84 ms, 2: 0.94, 4: 0.51, 8: 0.42, 16: see there
        static const int v = [] { const char *e = diag_env("MPFFT_CB_V"); const int x = e ? atoi(e) : 8;
                                  return x == 1 || x == 2 || x == 4 || x == 16 ? x : 8; }();
        return v;
    }
    // k_combine1's form for plan P: consecutive limbs per thread (combine.hpp) where a wave's 512
    // limbs meet at most 4 coefficients, else the per-limb form (MPFFT_COMB_CT = 0: per-limb, A/B)
    static int comb_kw(const Plan &P) { return (int)((P.N + 32767) / P.bits1 + 1); }
    static bool comb_ct(const Plan &P)
    {
        static const bool no_ct = [] { const char *e = diag_env("MPFFT_COMB_CT"); return e && !strcmp(e, "0"); }();
        return comb_v() == 8 && !no_ct && comb_kw(P) <= 4;
    }
    // threads per k_combine1 block: 512 for the consecutive form (C3 combine 0.285 -> 0.266 ms
    // against 256, profiles/r05/combine_ct_ab.txt; MPFFT_COMB_NT = 256 for A/B), 256 per-limb
    static int comb_nt(const Plan &P)
    {
        static const int nt = [] { const char *e = diag_env("MPFFT_COMB_NT"); return e && atoi(e) == 256 ? 256 : 512; }();
        return comb_ct(P) ? nt : 256;
    }
    static long comb_blocks(const Plan &P, long mcount)
    {
        const long bl = (long)comb_nt(P) * comb_v();
        return (mcount + bl - 1) / bl;
    }
    u32 *comb_flags(unsigned char *ws) const { return (u32 *)(ws + P.off_flags); }
    static long comb_flag_words(const Plan &P, long mcount) { return (comb_blocks(P, mcount) + 4) / 4 * 4; }

    // single-GPU workspace: both layouts are the natural one
    void single(unsigned char *ws)
    {
        col.dig[0] = (u64 *)(ws + P.off_digA);
        col.top[0] = (int *)(ws + P.off_topA);
        col.cb[0] = (u64 *)(ws + P.off_cbA);
        col.dig[1] = (u64 *)(ws + P.off_digB);
        col.top[1] = (int *)(ws + P.off_topB);
        col.cb[1] = (u64 *)(ws + P.off_cbB);
        row = col;
        if (P.has_c) {
            cview.dig[0] = (u64 *)(ws + P.off_digC);
            cview.top[0] = (int *)(ws + P.off_topC);
            cview.cb[0] = (u64 *)(ws + P.off_cbC);
        }
        c0 = 0;
        ccount = (int)P.NC;
        r0 = 0;
        rcount = (int)P.Tr;
        ccb = (int)P.NC;
        cbb = P.lbC;
        cbs = (long)P.Tr * P.NC;
    }

    // both layouts start `slots` slots further on (the sqrt2 plan's second half)
    void shift(long slots)
    {
        const long cbw = cb_words((int)P.l);
        for (int k = 0; k < 2; ++k) {
            col.dig[k] += slots * P.l;
            col.cb[k] += slots * cbw;
            col.top[k] += slots;
        }
        row = col;
        if (cview.dig[0]) {
            cview.dig[0] += slots * P.l;
            cview.cb[0] += slots * cbw;
            cview.top[0] += slots;
        }
    }

    // rotation staging buffers for a G-coefficient pass: as many as fit in 64 KiB
    int stage_bufs(int G) const
    {
        long fit = (64L * 1024) / (16L * P.l);
        if (fit < 1) fit = 1;
        return (int)(fit < G ? fit : G);
    }

    // k_rpass takes a pass unless it needs a canonical store, has zero inputs outside the
    // split, or some level rotation is not a whole number of limb pairs
    int rpass_mode(const PassArgs &a, int logg, int dir) const
    {
        if (!P.rpass || logg > (dir ? rp_maxlogg_dit((int)P.l) : rp_maxlogg_fwd4((int)P.l)) || a.canon || a.rho % 128) return -1;
        if (dir == 0) {
            if (a.scale_e || a.tw_mode == 2) return -1;
            if (a.src[0] || a.src[1]) return a.tw_mode || a.pcarry ? -1 : 2;
            if (a.zero_from < (1 << a.lbM)) return -1;
            if (a.tw_mode == 1) return a.pcarry ? -1 : 1;
            return a.pcarry ? 3 : 0;
        }
        if (a.tw_mode == 1) return -1;
        const bool ltw = a.tw_mode == 3, hl = a.lvl0 + logg == a.lbM;   // 3: the inverse twiddle on load (it takes scale_e too)
        if (ltw && !hl) return -1;
        const int gx = !ltw && (a.tw_mode == 2 || a.scale_e) ? 1 : 0;
        if (a.fill_off && gx) return -1;
        return gx | (hl ? 2 : 0) | (a.fill_off ? 4 : 0) | (ltw ? 8 : 0);
    }

    // the k_rpass mode pass() launches for these arguments, -1: another kernel family
    int rp_mode(const PassArgs &a, int logg, int dir) const
    {
        int rm = rpass_mode(a, logg, dir);
        static const int rmask = [] { const char *e = diag_env("MPFFT_RPASS_OFF"); return e ? atoi(e) : 0; }();
        if (rm >= 0 && (rmask >> (4 * dir + rm) & 1)) rm = -1;   // diagnostics: bit 4 dir + mode off
        return rm;
    }

    // levels of a pass whose arguments mk(k) builds: k, unless k_rpass declines that pass and
    // k_bpass cannot hold 2^k coefficients in LDS (k_rpass takes more levels per pass than
    // k_bpass fits: three at l = 4096, four inverse at l = 2048) -- then k_bpass's limit
    template <typename MK>
    int fit(int k, int dir, MK mk) const
    {
        if (!P.big || !P.bp_lg || k <= P.bp_lg || rp_mode(mk(k), k, dir) >= 0) return k;
        return P.bp_lg;
    }

    // the groups a pass launches: all 2^(lbM - logg) per sub-array, except in a forward pass, where
    // only blocks of 2^(lbM - lvl0) positions meeting [need_lo, need) are live -- the kernels return
    // at once for the others, but a launched-and-returning 1024-thread workgroup with 147 KB of LDS
    // still cost C3's second column pass 0.3 ms (931 -> 636 us, profiles/r06/live_groups_ab.txt):
    // the grid covers [grp0, grp0 + ngroups) only
    static void live_groups(PassArgs &a, int logg, int dir)
    {
        a.ngroups = 1 << (a.lbM - logg);
        a.grp0 = 0;
        if (dir != 0) return;
        const int slg = a.lbM - a.lvl0, lobits = slg - logg;
        const long nh = 1L << a.lvl0;
        const long hlo = std::min<long>(nh, a.need_lo > 0 ? (long)a.need_lo >> slg : 0);
        const long hhi = std::min<long>(nh, ((long)a.need + (1L << slg) - 1) >> slg);
        if (hhi > hlo) {
            a.grp0 = (int)(hlo << lobits);
            a.ngroups = (int)((hhi - hlo) << lobits);
        }
    }

    int pass(PassArgs a, int logg, int dir, int nops)
    {
        const int rm = rp_mode(a, logg, dir);
        if (rm >= 0) {
            rp_fn f = rp_get((int)P.l, logg, dir, rm);
            if (!f) return MPFFT_EUNSUPPORTED;
            static const size_t pad = [] { const char *e = diag_env("MPFFT_RPASS_LDSPAD"); return e ? (size_t)atol(e) : 0; }();
            static const int abl = [] { const char *e = diag_env("MPFFT_ABLATE"); return e ? atoi(e) : 0; }();
            a.ablate = abl;
            const size_t lds = rp_lds((int)P.l, logg) + pad;   // pad: diagnostics (one workgroup per CU)
            allow_lds((const void *)f, lds);
            live_groups(a, logg, dir);
            dim3 grid((unsigned)((long)a.nsub * a.ngroups), (unsigned)nops);
            static const bool stamps = diag_env("MPFFT_RP_STAMPS") != nullptr;
            const unsigned nt = (unsigned)rp_nt((int)P.l, logg, dir);
            if (stamps) return bp_stamped(f, grid, nt, lds, a, logg, dir);
            hipLaunchKernelGGL(f, grid, dim3(nt), lds, s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.big) {
            // limb-aligned kernel unless some rotation of the pass has a sub-limb part
            const bool gen = (a.rho % 64) || (a.tw_mode && a.tw_w % 64) || (a.scale_e % 64);
            bp_fn f = gen ? bp_get_gen(logg, dir) : bp_get(logg, dir);
            if (!f) return MPFFT_EUNSUPPORTED;
            const size_t lds = bp_lds_need((int)P.l, 1 << logg);
            allow_lds((const void *)f, lds);
            live_groups(a, logg, dir);
            dim3 grid((unsigned)((long)a.nsub * a.ngroups), (unsigned)nops);
            const unsigned nthr = (unsigned)(64 * bp_waves((int)P.l, logg));
            static const bool stamps = diag_env("MPFFT_BP_STAMPS") != nullptr;
            if (stamps) return bp_stamped(f, grid, nthr, lds, a, logg, dir);
            hipLaunchKernelGGL(f, grid, dim3(nthr), lds, s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.wave && P.lds) {
            pass_fn f = wv_fns(P.wU, P.wfull).lpass(logg, dir);
            if (!f) return MPFFT_EUNSUPPORTED;
            const size_t lds = ((size_t)16 * P.l) << logg;
            allow_lds((const void *)f, lds);
            live_groups(a, logg, dir);
            dim3 grid((unsigned)((long)a.nsub * a.ngroups), (unsigned)nops);
            hipLaunchKernelGGL(f, grid, dim3(32 << logg), lds, s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.wave) {
            {
                const char *e = diag_env("MPFFT_ABLATE");
                a.ablate = e ? atoi(e) : 0;
            }
            pass_fn f = wv_fns(P.wU, P.wfull).pass(logg, dir);
            if (!f) return MPFFT_EUNSUPPORTED;
            const size_t lds = wpass_lds(P.wU, 1 << logg, (int)P.l);
            allow_lds((const void *)f, lds);
            live_groups(a, logg, dir);
            const long waves = (long)a.nsub * a.ngroups;
            dim3 grid((unsigned)((waves + WPB - 1) / WPB), (unsigned)nops);
            hipLaunchKernelGGL(f, grid, dim3(64 * WPB), lds, s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        pass_fn f = get_pass(P.U, logg, dir);
        if (!f) return MPFFT_EUNSUPPORTED;
        const int G = 1 << logg;
        const int rb = stage_bufs(G);
        const size_t lds_pass = lds_bytes((int)P.l, rb, G, P.U, nw);
        allow_lds((const void *)f, lds_pass);
        a.nbuf = rb;
        live_groups(a, logg, dir);
        dim3 grid((unsigned)((long)a.nsub * a.ngroups), (unsigned)nops);
        hipLaunchKernelGGL(f, grid, dim3(P.tpb), lds_pass, s, a);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    // diagnostics only (MPFFT_BP_STAMPS): run one k_bpass launch with per-workgroup phase
    // stamps and print the average phase lengths (s_memtime ticks) of the working groups
    int bp_stamped(bp_fn f, dim3 grid, unsigned nthr, size_t lds, PassArgs a, int logg, int dir)
    {
        const size_t nwg = (size_t)grid.x * grid.y;
        unsigned long long *d = nullptr;
        HIPCHK(hipMalloc((void **)&d, nwg * 64));
        HIPCHK(hipMemsetAsync(d, 0, nwg * 64, s));
        a.dbg = d;
        hipLaunchKernelGGL(f, grid, dim3(nthr), lds, s, a);
        HIPCHK(hipGetLastError());
        unsigned long long *h = (unsigned long long *)malloc(nwg * 64);
        HIPCHK(hipMemcpyAsync(h, d, nwg * 64, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        double sum[8] = {0};
        long cnt = 0;
        unsigned long long t0 = ~0ull, t1 = 0;
        for (size_t w = 0; w < nwg; ++w) {
            const unsigned long long *q = h + 8 * w;
            if (!q[7]) continue;   // skipped group (past the truncation point)
            ++cnt;
            if (q[0] < t0) t0 = q[0];
            if (q[7] > t1) t1 = q[7];
            unsigned long long prev = q[0];
            for (int k = 1; k < 8; ++k)
                if (q[k]) { sum[k] += (double)(q[k] - prev); prev = q[k]; }
        }
        fprintf(stderr, "%s logg=%d dir=%d l=%ld groups=%ld/%zu span=%llu ticks: load %.0f lv0 %.0f lv1 %.0f lv2 %.0f fin %.0f canon/hx %.0f store %.0f\n", nthr == RP_NT || nthr == 1024 ? "rp_stamps" : "bp_stamps",
                logg, dir, P.l, cnt, nwg, t1 - t0, sum[1] / cnt, sum[2] / cnt, sum[3] / cnt, sum[4] / cnt, sum[5] / cnt,
                sum[6] / cnt, sum[7] / cnt);
        free(h);
        (void)hipFree(d);
        return MPFFT_OK;
    }

    PassArgs base_args(const View &v) const
    {
        PassArgs a;
        memset(&a, 0, sizeof(a));
        for (int k = 0; k < 2; ++k) {
            a.dig[k] = v.dig[k];
            a.cb[k] = v.cb[k];
            a.top[k] = v.top[k];
        }
        a.bits1 = P.bits1;
        a.N = P.N;
        a.l = (int)P.l;
        a.pbb = 30;
        a.jNC = P.NC;
        return a;
    }

    // column layout passes over this rank's ccount columns
    PassArgs col_args() const
    {
        PassArgs a = base_args(col);
        a.sub_stride = 1;
        a.pos_stride = ccount;
        a.nsub = ccount;
        a.sub_off = c0;
        return a;
    }

    // row layout passes over this rank's rcount rows
    PassArgs row_args() const
    {
        PassArgs a = base_args(row);
        a.lbM = P.lbC;
        a.rho = (u64)P.w * P.NR;
        a.sub_stride = ccb;
        a.pos_stride = 1;
        a.pbb = cbb;
        a.pbs = cbs;
        a.nsub = rcount;
        a.sub_off = r0;
        a.zero_from = (int)P.NC;
        a.need = (int)P.NC;
        a.tw_w = (u64)P.w;
        a.tw_lbR = P.lbR;
        return a;
    }

    // stage 1: split + forward truncated column DIF (length NR, root 2^(w NC))
    // operand `op` alone (0 or 1) in slot 0 of the pass arguments, one grid row (nops = 1);
    // op < 0: both operands (grid rows 0, 1)
    static PassArgs only(PassArgs a, int op)
    {
        if (op == 1) {
            a.dig[0] = a.dig[1];
            a.cb[0] = a.cb[1];
            a.top[0] = a.top[1];
            a.src[0] = a.src[1];
            a.nsrc[0] = a.nsrc[1];
        }
        return a;
    }

    // Pending exponents across forward passes (carry_pend): a k_rpass DIF pass whose successor
    // in the same transform is also a k_rpass DIF pass skips its closing rotation round (the
    // last level's pending exponents, one LDS round trip of all G coefficients) and leaves them
    // in HBM; the successor folds them into its first level's partner rotations
    // (PassArgs::pcarry).  Nothing crosses a stage: the last pass of a transform owes nothing.
    PassArgs col_pass_args(int lvl) const
    {
        PassArgs a = col_args();
        a.zero_from = (int)P.NR;
        a.lbM = P.lbR;
        a.lvl0 = lvl;
        a.rho = (u64)P.w * P.NC;
        a.need = (int)P.Tr;
        if (own_hi > 0) {   // only rows [own_lo, own_hi) wanted: skip the DIF subtrees outside them
            a.need = own_hi < a.need ? own_hi : a.need;
            a.need_lo = own_lo;
        }
        return a;
    }

    int fwd_columns(const u64 *srcA, long nA, const u64 *srcB, long nB, int nops, int op = -1)
    {
        int lvl = 0, pend0 = 0;   // the data owe the pending exponents of levels [pend0, lvl)
        while (lvl < P.lbR) {
            PassArgs a = col_pass_args(lvl);
            if (lvl == 0) {
                a.src[0] = srcA; a.nsrc[0] = nA;
                a.src[1] = srcB; a.nsrc[1] = nB;
                a.src_chunk = src_chunk;
                a.zero_from = in_rows ? in_rows : (int)P.Tr;
                a.zp = zflags;
                a.zn = zflags_n;
            }
            if (op == 1) a.zp = nullptr;   // the combine flags are cleared by operand 0's pass
            a.pcarry = lvl - pend0;
            const int k = fit(split(P.lbR - lvl, true), 0, [&](int) { return a; });
            if (carry_pend && rp_mode(a, k, 0) >= 0 && (carry_mask() & 1) && lvl + k < P.lbR) {
                const int k2 = split(P.lbR - lvl - k, true);
                PassArgs n = col_pass_args(lvl + k);
                n.pcarry = k;   // it would owe this pass's levels
                a.pkeep = rp_mode(n, k2, 0) >= 0;
            }
            int rc = op < 0 ? pass(a, k, 0, nops) : pass(only(a, op), k, 0, 1);
            if (rc) return rc;
            // a keeping pass owes its own levels only (a receiving pass applies what it was
            // owed on load: rotated load, k_rpass MODE 3)
            pend0 = a.pkeep ? lvl : lvl + k;
            lvl += k;
        }
        return MPFFT_OK;
    }

    // the last row level fused into k_pwss: slot pairs (2i, 2i + 1) of a row adjacent (any row
    // layout with column blocks of ccb >= 2), a nested negacyclic pointwise with its fused-pair
    // instance, and a row pass left to apply the MFA twiddle
    // row DIF levels fused into the pointwise (0, 1 or 2)
    int row_fused() const
    {
        static const bool off = [] { const char *e = diag_env("MPFFT_FUSE_ROW"); return e && !strcmp(e, "0"); }();
        const int f = P.fuse_rows;
        return fuse_row_last && !off && f && cview.dig[0] && pw_pair_kernel(P.l, f) && ccb >= (1 << f) ? f : 0;
    }

    int row_levels() const { return P.lbC - row_fused(); }

    PassArgs row_pass_args(int lvl, int k, int L) const
    {
        PassArgs a = row_args();
        a.lvl0 = lvl;
        a.tw_mode = lvl == 0 ? 1 : 0;
        // canonical pointwise inputs, except for k_pwss (it loads the reduced form)
        if (lvl + k == L) a.canon = pwss_active() ? 0 : 1;
        return a;
    }

    // stage 2: MFA twiddle + row DIF (length NC, root 2^(w NR)), canonical out
    int fwd_rows(int nops, int op = -1)
    {
        int lvl = 0, pend0 = 0;
        const int L = row_levels();
        while (lvl < L) {
            auto mk = [&](int kk) {
                PassArgs b = row_pass_args(lvl, kk, L);
                b.pcarry = lvl - pend0;
                return b;
            };
            const int k = fit(split(L - lvl), 0, mk);
            PassArgs a = mk(k);
            if (carry_pend && (carry_mask() & 4) && lvl + k < L && rp_mode(a, k, 0) >= 0) {
                const int k2 = split(L - lvl - k);
                PassArgs n = row_pass_args(lvl + k, k2, L);
                n.pcarry = k;   // it would owe this pass's levels
                a.pkeep = rp_mode(n, k2, 0) >= 0;
            }
            int rc = op < 0 ? pass(a, k, 0, nops) : pass(only(a, op), k, 0, 1);
            if (rc) return rc;
            // a keeping pass owes its own levels only (a receiving pass applies what it was
            // owed on load: rotated load, k_rpass MODE 3)
            pend0 = a.pkeep ? lvl : lvl + k;
            lvl += k;
        }
        return MPFFT_OK;
    }

    // nested negacyclic pointwise (pkernels.hpp) for big coefficients: (l -> pieces 2^lk)
  public:
    static int pwss_lk(long l) { return pwss_lk_of(l); }

    bool pwss_active() const
    {
        const int lk = pwss_lk(P.l);
        return lk && pw_get(pw_inner_limbs(P.l, lk), lk) != nullptr;
    }

    long pw_count = 0;   // > 0: the pointwise covers this many slots from the row views (a row chunk of one column block)

    int pointwise()
    {
        const long cnt = pw_count > 0 ? pw_count : (long)rcount * P.NC;
        if (cnt == 0) return MPFFT_OK;
        if (const int lk = pwss_lk(P.l)) {
            const int M = pw_inner_limbs(P.l, lk);
            const int fz = row_fused();
            const bool pair = fz > 0;
            pw_fn f = pw_get(M, lk, fz);
            if (f) {
                const size_t lds = pw_lds(M, 1 << lk, (int)P.l);
                allow_lds((const void *)f, lds);
                static const bool stamps = diag_env("MPFFT_PW_STAMPS") != nullptr;
                unsigned long long *dbg = nullptr;
                if (stamps) {   // diagnostics only: per-workgroup phase stamps, averaged on the host
                    HIPCHK(hipMalloc((void **)&dbg, (size_t)cnt * 64));
                    HIPCHK(hipMemsetAsync(dbg, 0, (size_t)cnt * 64, s));
                }
                hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(1u << lk), lds, s, row.dig[0], row.cb[0], row.top[0],
                                   (const u64 *)row.dig[1], (const u64 *)row.cb[1], (const int *)row.top[1], (int)P.l,
                                   cview.dig[0], cview.cb[0], cview.top[0], dbg);
                HIPCHK(hipGetLastError());
                if (pair) {   // the product lives in C from here on (single layout: rows == columns)
                    row.dig[0] = col.dig[0] = cview.dig[0];
                    row.cb[0] = col.cb[0] = cview.cb[0];
                    row.top[0] = col.top[0] = cview.top[0];
                }
                if (stamps) {
                    unsigned long long *h = (unsigned long long *)malloc((size_t)cnt * 64);
                    HIPCHK(hipMemcpyAsync(h, dbg, (size_t)cnt * 64, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipStreamSynchronize(s));
                    double sum[8] = {0};
                    long n = 0;
                    for (long w = 0; w < cnt; ++w) {
                        const unsigned long long *q = h + 8 * w;
                        if (!q[7]) continue;
                        ++n;
                        for (int k = 1; k < 8; ++k) sum[k] += (double)(q[k] - q[k - 1]);
                    }
                    fprintf(stderr, "pw_stamps M=%d lk=%d slots=%ld/%ld: load %.0f fwdA %.0f fwdB %.0f mul %.0f inv %.0f final %.0f out %.0f\n",
                            M, lk, n, cnt, sum[1] / n, sum[2] / n, sum[3] / n, sum[4] / n, sum[5] / n, sum[6] / n, sum[7] / n);
                    free(h);
                    (void)hipFree(dbg);
                }
                return MPFFT_OK;
            }
        }
        static const long pwm2_maxl = [] { const char *e = diag_env("MPFFT_PWM2_MAXL"); return e ? atol(e) : 4096L; }();
        if (P.l % 256 == 0 && P.l <= pwm2_maxl && pw_kind() != PW_MFMA1 && pw_kind() != PW_VALU) {   // int8 MFMA, register-blocked: 2 fold tiles per wave
            const int nw = (int)P.l / 256;
            const int tpb = 64 * nw;
            const size_t lds = pwm_lds_bytes((int)P.l, 4, nw);
            void (*f)(u64 *, u64 *, int *, const u64 *, const int *, int, int) =
                diag_env("MPFFT_PWM2_D4") && nw <= 8 ? k_pwm2<4, 2, 4> : k_pwm2<4, 2, 2>;   // D = 4: more VGPRs, slower at C2
            const char *ea = diag_env("MPFFT_PWABLATE");   // timing experiments only: 1 = no MFMA phase
            allow_lds((const void *)f, lds);
            hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(tpb), lds, s, row.dig[0], row.cb[0], row.top[0],
                               (const u64 *)row.dig[1], (const int *)row.top[1], (int)P.l, ea ? atoi(ea) : 0);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.l % 128 == 0 && pw_kind() != PW_VALU) {   // int8 MFMA Toeplitz product
            const int nw = std::min((int)P.l / 128, 16);
            const int tpb = 64 * nw;
            const int U = (int)P.l / tpb;
            const size_t lds = pwm_lds_bytes((int)P.l, U, nw);
            void (*f)(u64 *, u64 *, int *, const u64 *, const int *, int) = nullptr;
            if (U == 2) f = k_pwm<2, 1>;
            else if (U == 4) f = k_pwm<4, 2>;
            else return MPFFT_EUNSUPPORTED;
            allow_lds((const void *)f, lds);
            hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(tpb), lds, s, row.dig[0], row.cb[0], row.top[0],
                               (const u64 *)row.dig[1], (const int *)row.top[1], (int)P.l);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.l % 2 == 0 && P.l >= 32) {   // register-blocked kernel: R columns per thread
            const int R = P.l >= 2048 ? 8 : 4;
            const int L = 2 * (int)P.l;
            const int tpb = (L / R + 63) / 64 * 64;   // whole waves (threads past L/R idle in the MAC loop)
            const size_t lds = (size_t)3 * L * 4 + (norm_scr_u64(1, R / 2, 16) + 2) * 8;
            void (*f)(u64 *, u64 *, int *, const u64 *, const int *, int) = R == 8 ? k_pw<8> : k_pw<4>;
            allow_lds((const void *)f, lds);
            hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(tpb), lds, s, row.dig[0], row.cb[0], row.top[0],
                               (const u64 *)row.dig[1], (const int *)row.top[1], (int)P.l);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        const size_t lds = (size_t)3 * 2 * P.l * 4 + (norm_scr_u64(1, P.U, 16) + 2) * 8;
        void (*f)(u64 *, u64 *, int *, const u64 *, const int *, int, u64) = nullptr;
        switch (P.U) {
        case 1: f = k_pointwise<1>; break;
        case 2: f = k_pointwise<2>; break;
        case 4: f = k_pointwise<4>; break;
        }
        allow_lds((const void *)f, lds);
        hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(P.tpb), lds, s, row.dig[0], row.cb[0], row.top[0],
                           (const u64 *)row.dig[1], (const int *)row.top[1], (int)P.l, P.N);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    // stage 4: row DIT inverse, MFA un-twiddle at the end
    int inv_rows()
    {
        int hi = P.lbC;
        while (hi > 0) {
            auto mk = [&](int kk) {
                PassArgs b = row_args();
                b.lvl0 = hi - kk;
                b.tw_mode = (hi - kk == 0 && !(fold && P.ltw)) ? 2 : 0;   // (ltw: on load in the column blocks)
                if (fold && !P.ltw && hi - kk == 0) b.scale_e = 2 * P.N - (u64)(P.depth + 1);   // the scaling rides in the un-twiddle
                return b;
            };
            const int k = fit(split(hi, false, true), 1, mk);
            PassArgs a = mk(k);
            int rc = pass(a, k, 1, 1);
            if (rc) return rc;
            hi -= k;
        }
        return MPFFT_OK;
    }

    // full inverse (DIT) over block [off, off + m) of every local column
    int ifft_block(long off, long m)
    {
        if (int rc = flush_chain()) return rc;
        const int lbM = ilog2(m);
        int hi = lbM;
        while (hi > 0) {
            auto mk = [&](int kk) {
                PassArgs b = col_args();
                b.lbM = lbM;
                b.lvl0 = hi - kk;
                b.rho = rho_blk(m);
                b.pos_off = (int)off;
                b.zero_from = (int)m;
                b.need = (int)m;
                if (P.fuse_scale && hi - kk == 0 && m == P.NR) {   // the whole column inverse is this block
                    b.scale_e = 2 * P.N - (u64)(P.depth + 1);
                    b.canon = 1;
                }
                if (fold && P.ltw && hi == lbM) {   // the block's first pass: inverse MFA twiddle + scaling on load
                    b.tw_mode = 3;
                    b.tw_w = (u64)P.w;
                    b.tw_lbR = P.lbR;
                    b.scale_e = 2 * P.N - (u64)(P.depth + 1);
                }
                return b;
            };
            const int k = fit(split(hi, true, true), 1, mk);
            PassArgs a = mk(k);
            if (hi - k == 0 && fill.off) {   // the block's last pass also does the pending FILL step
                PassArgs f = a;
                f.fill_lo = (int)fill.lo;
                f.fill_off = (int)fill.off;
                f.fill_rho = fill.rho;
                if (rp_mode(f, k, 1) >= 0) {
                    a = f;
                    fill.done = true;
                }
            }
            int rc = pass(a, k, 1, 1);
            if (rc) return rc;
            hi -= k;
        }
        return MPFFT_OK;
    }

    // The truncated inverse's tail (Exec::chain): TWOXMY steps on one row range are held back
    // and run together with the IBFLY that consumes their rows (k_rchain), so those rows are
    // read once; anything else flushes them first.
    struct Chain { long off = 0, t = 0; int n = 0; long h[3] = {0, 0, 0}; } chain;

    int flush_chain()
    {
        const Chain c = chain;
        chain.n = 0;
        for (int j = 0; j < c.n; ++j) {
            int rc = pairop_now(OP_TWOXMY, c.off, c.h[j], 0, c.t, 0);
            if (rc) return rc;
        }
        return MPFFT_OK;
    }

    PairArgs pair_args(int op, long off, long h, long i0, long cnt, u64 rho) const
    {
        PairArgs a;
        memset(&a, 0, sizeof(a));
        a.dig = col.dig[0];
        a.cb = col.cb[0];
        a.top = col.top[0];
        a.N = P.N;
        a.l = (int)P.l;
        a.op = op;
        a.NC = ccount;
        a.ncol = ccount;
        a.off = (int)off;
        a.h = (int)h;
        a.i0 = (int)i0;
        a.cnt = (int)cnt;
        a.rho = rho;
        return a;
    }

    int pairop(int op, long off, long h, long i0, long cnt, u64 rho)
    {
        if (cnt <= 0) return MPFFT_OK;
        int rc;
        const bool chains = P.rpass && rp_chain_get((int)P.l, 1) && !diag_env("MPFFT_NO_CHAIN");
        if (chains && op == OP_TWOXMY && i0 == 0) {
            if (chain.n && (chain.off != off || chain.t != cnt || chain.n == 3) && (rc = flush_chain())) return rc;
            if (!chain.n) {
                chain.off = off;
                chain.t = cnt;
            }
            chain.h[chain.n++] = h;
            return MPFFT_OK;
        }
        if (chains && op == OP_IBFLY && i0 == 0 && chain.n && chain.off == off + h && chain.t == cnt) {
            PairArgs a = pair_args(op, off + h, h, 0, cnt, rho);
            a.nb = chain.n;
            for (int j = 0; j < chain.n; ++j) a.hb[j] = (int)chain.h[j];
            a.xoff = (int)off;
            rp_pair_fn f = rp_chain_get((int)P.l, chain.n);
            chain.n = 0;
            hipLaunchKernelGGL(f, dim3((unsigned)(cnt * ccount)), dim3(RP_NT), rp_chain_lds((int)P.l), s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if ((rc = flush_chain())) return rc;
        return pairop_now(op, off, h, i0, cnt, rho);
    }

    int pairop_now(int op, long off, long h, long i0, long cnt, u64 rho)
    {
        if (cnt <= 0) return MPFFT_OK;
        PairArgs a;
        a.dig = col.dig[0];
        a.cb = col.cb[0];
        a.top = col.top[0];
        a.N = P.N;
        a.l = (int)P.l;
        a.op = op;
        a.NC = ccount;
        a.ncol = ccount;
        a.off = (int)off;
        a.h = (int)h;
        a.i0 = (int)i0;
        a.cnt = (int)cnt;
        a.rho = rho;
        if (P.rpass) {   // register-resident pair steps (rkernels.hpp)
            rp_pair_fn f = rp_pair_get((int)P.l, op);
            if (!f) return MPFFT_EUNSUPPORTED;
            hipLaunchKernelGGL(f, dim3((unsigned)(cnt * ccount)), dim3(RP_NT), rp_pair_lds((int)P.l), s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.wave) {
            void (*f)(PairArgs) = wv_fns(P.wU, P.wfull).pair;
            const size_t lds = (size_t)WPB * 16 * P.l;
            allow_lds((const void *)f, lds);
            const long waves = cnt * ccount;
            hipLaunchKernelGGL(f, dim3((unsigned)((waves + WPB - 1) / WPB)), dim3(64 * WPB), lds, s, a);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        const size_t lds = lds_bytes((int)P.l, 2, 2, P.U, nw);
        void (*f)(PairArgs) = nullptr;
        switch (P.U) {
        case 1: f = k_pairop<1>; break;
        case 2: f = k_pairop<2>; break;
        case 4: f = k_pairop<4>; break;
        }
        allow_lds((const void *)f, lds);
        hipLaunchKernelGGL(f, dim3((unsigned)(cnt * ccount)), dim3(P.tpb), lds, s, a);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    u64 rho_blk(long m) const { return (u64)P.w * P.NC * (u64)(P.NR / m); }

    // IFFT_radix2_truncate(_twiddle) (mul_fft.c:1733-1790): outputs [off, off+t) known,
    // inputs >= t zero; root of a length-m block = 2^(w NC NR/m)
    // public entries: the recursion, then whatever it left in the chain
    int itft(long off, long m, long t)
    {
        int rc = itft_r(off, m, t);
        return rc ? rc : flush_chain();
    }
    int itft1(long off, long m, long t)
    {
        int rc = itft1_r(off, m, t);
        return rc ? rc : flush_chain();
    }

    int itft_r(long off, long m, long t)
    {
        int rc;
        const long h = m / 2;
        const bool top = defer_double && off == 0 && m == P.NR;   // its doubling folds into the scaling
        if (t == m) return ifft_block(off, m);
        if (t <= h) {
            if ((rc = itft_r(off, h, t))) return rc;
            if (top) {
                dbl_lo = 0;
                dbl_hi = t;
                return MPFFT_OK;
            }
            return pairop(OP_DOUBLE, off, h, 0, t, 0);
        }
        fill = {t - h, h, rho_blk(m), false};   // offered to ifft_block's last pass
        rc = ifft_block(off, h);
        const bool filled = fill.done;
        fill = {};
        if (rc) return rc;
        if (!filled && (rc = pairop(OP_FILL, off, h, t - h, h - (t - h), rho_blk(m)))) return rc;
        if ((rc = itft1_r(off + h, h, t - h))) return rc;
        if ((rc = pairop(OP_IBFLY, off, h, 0, t - h, rho_blk(m)))) return rc;
        if (top) {
            dbl_lo = t - h;
            dbl_hi = h;
            return MPFFT_OK;
        }
        return pairop(OP_DOUBLE, off, h, t - h, h - (t - h), 0);
    }

    // IFFT_radix2_truncate1(_twiddle) (mul_fft.c:1604-1668): inputs [t, m) known
    int itft1_r(long off, long m, long t)
    {
        int rc;
        const long h = m / 2;
        if (t == m) return ifft_block(off, m);
        if (t <= h) {
            if ((rc = pairop(OP_HALFADD, off, h, t, h - t, 0))) return rc;
            if ((rc = itft1_r(off, h, t))) return rc;
            return pairop(OP_TWOXMY, off, h, 0, t, 0);
        }
        if ((rc = ifft_block(off, h))) return rc;
        if ((rc = pairop(OP_FIX, off, h, t - h, h - (t - h), rho_blk(m)))) return rc;
        if ((rc = itft1_r(off + h, h, t - h))) return rc;
        return pairop(OP_IBFLY, off, h, 0, t - h, rho_blk(m));
    }

    // scaling by 2^-(depth+1); rows [dbl_lo, dbl_hi) by 2^-depth (itft's deferred doubling)
    int scale()
    {
        if (P.fuse_scale || fold) return MPFFT_OK;   // done by the last inverse column / row pass
        const u64 e = 2 * P.N - (u64)(P.depth + 1);
        if (dbl_hi <= dbl_lo) return scale_rows(0, P.Tr, e);
        if (P.rpass) return scale_rows(0, P.Tr, e, dbl_lo, dbl_hi);   // one launch, two exponents
        int rc;
        if ((rc = scale_rows(0, dbl_lo, e))) return rc;
        if ((rc = scale_rows(dbl_lo, dbl_hi, e + 1))) return rc;
        return scale_rows(dbl_hi, P.Tr, e);
    }

    // rows [r0_, r1_) by 2^e; with rpass, rows [d0, d1) inside them by 2^(e+1)
    int scale_rows(long r0_, long r1_, u64 e, long d0 = 0, long d1 = 0)
    {
        const long cnt = (r1_ - r0_) * ccount, s0 = r0_ * ccount;
        if (cnt <= 0) return MPFFT_OK;
        u64 *dig = col.dig[0] + s0 * P.l, *cbp = col.cb[0] + s0 * cb_words((int)P.l);
        int *top = col.top[0] + s0;
        if (P.rpass) {   // register-resident scale + canonicalisation (rkernels.hpp)
            // threads per coefficient: 256 up to l = 2048 (C3 scale 0.36 -> 0.31 ms: more coefficients
            // in flight per CU), 512 at l = 4096 (C4 2.61 vs 2.96 ms: the canonical sweep's rows per
            // wave double); profiles/r03/scale_nt_ab.txt
            static const int snt_env = [] { const char *e = diag_env("MPFFT_SCALE_NT"); return e ? atoi(e) : 0; }();
            const int snt = snt_env == 256 || snt_env == 512 ? snt_env : P.l <= 2048 ? 256 : 512;
            rp_scale_fn f = rp_scale_get((int)P.l, snt);
            if (!f) return MPFFT_EUNSUPPORTED;
            const unsigned lo = (unsigned)((d0 - r0_) * ccount), hi = (unsigned)((d1 - r0_) * ccount);
            hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(snt), rp_scale_lds((int)P.l), s, dig, cbp, top, (unsigned)P.N,
                               (unsigned)e, (unsigned)(e + 1), d1 > d0 ? lo : 0u, d1 > d0 ? hi : 0u);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        if (P.wave) {
            wv_scale_fn f = wv_fns(P.wU, P.wfull).scale;
            const size_t lds = (size_t)WPB * 16 * P.l;
            allow_lds((const void *)f, lds);
            hipLaunchKernelGGL(f, dim3((unsigned)((cnt + WPB - 1) / WPB)), dim3(64 * WPB), lds, s, dig, cbp, top,
                               (int)P.l, P.N, e, cnt);
            HIPCHK(hipGetLastError());
            return MPFFT_OK;
        }
        const size_t lds = lds_bytes((int)P.l, 1, 1, P.U, nw);
        void (*f)(u64 *, u64 *, int *, int, u64, u64) = nullptr;
        switch (P.U) {
        case 1: f = k_scale<1>; break;
        case 2: f = k_scale<2>; break;
        case 4: f = k_scale<4>; break;
        }
        allow_lds((const void *)f, lds);
        hipLaunchKernelGGL(f, dim3((unsigned)cnt), dim3(P.tpb), lds, s, dig, cbp, top, (int)P.l, P.N, e);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    // combine stripes (combine.hpp): `a` names the coefficients, the stripes (a.G, a.g, a.S, a.C)
    // and the halo; nst stripes of this launch, each comb_blocks(stripe limbs) blocks, in one
    // k_combine1 launch (window sums plus a per-stripe decoupled look-back carry chain, carry-in
    // 0).  st: the look-back flags (nst bps + 1 u32, zeroed here unless `cleared`); allp (or
    // null): per-block all-ones flags for the stripe summaries.
    int combine1(CombArgs a, long nst, long stripe_limbs, u64 *r, u32 *st, bool cleared, u32 *allp)
    {
        a.l = (int)P.l;
        a.N = P.N;
        a.bits1 = P.bits1;
        a.len = P.len;
        a.total = P.total;
        a.inv_bits1 = 1.0 / (double)P.bits1;
        a.bps = comb_blocks(P, stripe_limbs);
        const long nb = nst * a.bps;
        if (!cleared) HIPCHK(hipMemsetAsync(st, 0, (size_t)(nb + 1) * 4, s));   // one fill
        const int v = comb_v();
        const bool k3 = (P.N + 63 + P.bits1 - 1) / P.bits1 <= 3;   // at most 3 coefficients cover a limb
        void (*f)(CombArgs, u64 *, u32 *, u32 *) =
            k3 ? (v == 1 ? k_combine1<1, 3> : v == 2 ? k_combine1<2, 3> : v == 4 ? k_combine1<4, 3>
                  : v == 16 ? k_combine1<16, 3> : k_combine1<8, 3>)
               : (v == 1 ? k_combine1<1, 0> : v == 2 ? k_combine1<2, 0> : v == 4 ? k_combine1<4, 0>
                  : v == 16 ? k_combine1<16, 0> : k_combine1<8, 0>);
        // consecutive limbs per thread: the wave's pairs loaded coalesced and handed out through LDS
        // (C3 combine 0.300 -> 0.285 ms against per-lane pair loads; MPFFT_COMB_XP = 0 for A/B)
        static const bool no_xp = [] { const char *e = diag_env("MPFFT_COMB_XP"); return e && !strcmp(e, "0"); }();
        const int nt = comb_nt(P);
        if (comb_ct(P)) {
            const bool k3w = comb_kw(P) <= 3;
            if (!no_xp) f = nt == 512 ? (k3w ? k_combine1<8, 3, true, 512, true> : k_combine1<8, 4, true, 512, true>)
                                      : (k3w ? k_combine1<8, 3, true, 256, true> : k_combine1<8, 4, true, 256, true>);
            else f = nt == 512 ? (k3w ? k_combine1<8, 3, true, 512> : k_combine1<8, 4, true, 512>)
                               : (k3w ? k_combine1<8, 3, true> : k_combine1<8, 4, true>);
        }
        hipLaunchKernelGGL(f, dim3((unsigned)nb), dim3(nt), 0, s, a, r, st, allp);   // st[nb]: the ticket counter
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    // f4: the combine from the reduced form (fold.hpp): k_cmeta, then k_combine_red; rows
    // [lo, hi) of the coefficients doubled
    int combine_fold(u64 *r, unsigned char *ws, long lo, long hi)
    {
        FoldArgs a;
        memset(&a, 0, sizeof(a));
        a.dig = row.dig[0];
        a.cb = row.cb[0];
        a.top = row.top[0];
        a.meta = (int *)(ws + P.off_meta);
        a.l = (int)P.l;
        a.cbw = cb_words((int)P.l);
        a.N = P.N;
        a.bits1 = P.bits1;
        a.len = P.len;
        a.total = P.total;
        a.lbC = P.lbC;
        a.dbl_lo = (int)lo;
        a.dbl_hi = (int)hi;
        a.inv_bits1 = 1.0 / (double)P.bits1;
        constexpr int NT = 512;
        a.bps = (P.total + 8 * NT - 1) / (8 * NT);
        u32 *st = comb_flags(ws);
        if (zflags != st) HIPCHK(hipMemsetAsync(st, 0, (size_t)(a.bps + 1) * 4, s));
        auto cm = P.l == 1024 ? k_cmeta<16> : P.l == 2048 ? k_cmeta<32> : P.l == 4096 ? k_cmeta<64> : k_cmeta<0>;
        hipLaunchKernelGGL(cm, dim3((unsigned)((P.len + 255) / 256)), dim3(256), 0, s, a);   // a lane per coefficient
        HIPCHK(hipGetLastError());
        void (*f)(FoldArgs, u64 *, u32 *) = P.fold == 3 ? k_combine_red<3, NT> : k_combine_red<4, NT>;
        // persistent grid: the resident block count (workgroups take tickets until none are left)
        long grid = a.bps;
        if (FOLD_PERSIST) {
            int per = 0, ncu = 0, dev = 0;
            if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess
                && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)f, NT, 0) == hipSuccess && per > 0 && ncu > 0)
                grid = std::min<long>(grid, (long)per * ncu);
        }
        hipLaunchKernelGGL(f, dim3((unsigned)grid), dim3(NT), 0, s, a, r, st);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }

    // one GPU: a single stripe over the natural slot order (coefficient k at slot k)
    int combine_single(u64 *r, unsigned char *ws)
    {
        u32 *st = comb_flags(ws);
        CombArgs a;
        memset(&a, 0, sizeof(a));
        a.dig = row.dig[0];
        a.C = P.trunc;
        a.G = 1;
        a.S = 1;
        return combine1(a, 1, P.total, r, st, zflags == st, nullptr);
    }
};

// Stage profiling (mpfft_profile_begin/end): while active, each multiply claims a call slot
// and records a HIP event on its own stream at every stage boundary -- the timed calls are
// otherwise unchanged -- and profile_end sums the per-stage times of the calls that
// recorded every boundary.  A claimed slot keeps its own event pointer (taken under the
// lock), and profile_begin refuses to reallocate while claimed calls are still running.
struct StageProf {
    bool on = false;
    int cap = 0, used = 0, inflight = 0;
    hipEvent_t *ev = nullptr;   // cap * (MPFFT_NSTAGES + 1)
    int *marks = nullptr;       // per claimed call: boundaries recorded (MPFFT_NSTAGES + 1 = complete)
};
static std::mutex g_prof_mu;
static StageProf g_prof;

struct ProfCall {
    int call = -1;
    hipEvent_t *ev = nullptr;
    int marks = 0;
    ProfCall()
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (g_prof.on && g_prof.used < g_prof.cap) {
            call = g_prof.used++;
            ev = g_prof.ev + (size_t)call * (MPFFT_NSTAGES + 1);
            ++g_prof.inflight;
        }
    }
    void mark(int stage, hipStream_t s)
    {
        if (call < 0) return;
        if (hipEventRecord(ev[stage], s) == hipSuccess && stage == marks) ++marks;
    }
    ~ProfCall()
    {
        if (call < 0) return;
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof.marks[call] = marks;
        --g_prof.inflight;
    }
};

// the sqrt2 top level (kernels.hpp k_s2op): one workgroup per k in [k0, k0 + cnt)
static int s2_launch(const Plan &P, const Exec &X, int op, const u64 *srcA, const u64 *srcB, long k0, long cnt,
                     long tlo, int nops)
{
    if (cnt <= 0) return MPFFT_OK;
    S2Args a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < 2; ++k) {
        a.dig[k] = X.col.dig[k];
        a.cb[k] = X.col.cb[k];
        a.top[k] = X.col.top[k];
    }
    a.src[0] = srcA; a.nsrc[0] = P.n1;
    a.src[1] = srcB; a.nsrc[1] = P.n2;
    a.bits1 = P.bits1;
    a.N = P.N;
    a.w = (u64)P.w;
    a.l = (int)P.l;
    a.op = op;
    a.half = 2 * P.n;
    a.k0 = k0;
    a.tlo = tlo;
    void (*f)(S2Args) = nullptr;
    // l = 2048: four limbs per thread over 512 threads (k_s2op<2> at 1024 threads spilled 388 B)
    const int U = P.U == 2 && P.l == 2048 && !diag_env("MPFFT_S2_U2") ? 4 : P.U;
    const int tpb = (int)(P.l / U) < P.tpb ? (int)(P.l / U) : P.tpb;
    switch (U) {
    case 1: f = k_s2op<1>; break;
    case 2: f = k_s2op<2>; break;
    case 4: f = k_s2op<4>; break;
    }
    if (!f) return MPFFT_EUNSUPPORTED;
    const size_t lds = lds_bytes((int)P.l, s2_rb(U), 3, U, tpb / 64);
    allow_lds((const void *)f, lds);
    hipLaunchKernelGGL(f, dim3((unsigned)cnt, (unsigned)nops), dim3(tpb), lds, X.s, a);
    HIPCHK(hipGetLastError());
    return MPFFT_OK;
}

// new_mpn_mul6 (mul_fft.c:3573-3668) on the GPU: the sqrt2 top level (k_s2op) around two
// length-2n MFA multiplies that reuse every stage of run_all -- the first half full, the
// second truncated to trunc2 = Tr - NR rows (FFT/IFFT_radix2_mfa_truncate_sqrt2 :2212, :2593)
static int run_all6(const Plan &P, u64 *d_r, const u64 *d_i1, const u64 *d_i2, unsigned char *ws, hipStream_t s)
{
    Plan P1 = P, P2 = P, PS = P;
    P1.Tr = P.NR;
    P1.trunc = 2 * P.n;
    P2.Tr = P.Tr > P.NR ? P.Tr - P.NR : 0;
    P2.trunc = P2.Tr * P.NC;
    PS.depth = P.depth + 1;   // scale by 2^-(depth+2) (:3654-3658)
    Exec X1(P1, s), X2(P2, s), XS(PS, s), XC(P, s);
    X1.single(ws);
    X2.single(ws);
    X2.shift(2 * P.n);
    X2.in_rows = (int)P.NR;   // the second half's inputs are all live (FFT_radix2_truncate1_twiddle)
    X1.fuse_row_last = X2.fuse_row_last = true;   // each half's last row level inside its pointwise
    XS.single(ws);
    XC.single(ws);
    const bool two = P2.Tr > 0;
    const long tlo = P.trunc - 2 * P.n;   // pairs k < tlo carry both halves
    int rc;
    ProfCall pc;   // stage events as run_all's (the sqrt2 top level counts with the columns)
    pc.mark(0, s);
    if ((rc = s2_launch(P, X1, S2_FWD, d_i1, d_i2, 0, 2 * P.n, two ? 1 : 0, 2))) return rc;
    if ((rc = X1.fwd_columns(nullptr, 0, nullptr, 0, 2))) return rc;
    if (two && (rc = X2.fwd_columns(nullptr, 0, nullptr, 0, 2))) return rc;
    pc.mark(1, s);
    if ((rc = X1.fwd_rows(2))) return rc;
    if (two && (rc = X2.fwd_rows(2))) return rc;
    pc.mark(2, s);
    const bool fused = X1.row_fused() > 0;
    if ((rc = X1.pointwise())) return rc;
    if (two && (rc = X2.pointwise())) return rc;
    pc.mark(3, s);
    if (fused) {   // the products (and everything after) live in C: X1's views now start there
        XS.col = XS.row = X1.col;
        XC.col = XC.row = X1.col;
    }
    if ((rc = X1.inv_rows())) return rc;
    if (two && (rc = X2.inv_rows())) return rc;
    pc.mark(4, s);
    if ((rc = X1.itft(0, P.NR, P.NR))) return rc;
    if (two) {
        if ((rc = s2_launch(P, X1, S2_FILL, nullptr, nullptr, P2.Tr * P.NC, (P.NR - P2.Tr) * P.NC, 0, 1))) return rc;
        if ((rc = X2.itft1(0, P.NR, P2.Tr))) return rc;
    }
    if ((rc = s2_launch(P, X1, S2_IBFLY, nullptr, nullptr, 0, 2 * P.n, tlo > 0 ? tlo : 0, 1))) return rc;
    pc.mark(5, s);
    if ((rc = XS.scale())) return rc;
    pc.mark(6, s);
    rc = XC.combine_single(d_r, ws);
    pc.mark(7, s);
    return rc;
}

// Host operands (mul_host): operand 2's copy from the host runs on the context's copy stream
// while operand 1's forward columns and rows run on `s`; operand 2's passes wait for it.
struct HostB {
    const u64 *h;       // host limbs of operand 2 (null: d_i2 is already on the device)
    hipStream_t cs;     // copy stream
    hipEvent_t ready;   // recorded on cs after the copy
};

static int run_all(const Plan &P, u64 *d_r, const u64 *d_i1, const u64 *d_i2, unsigned char *ws, hipStream_t s,
                   const HostB *hb = nullptr)
{
    if (P.sqrt2) return run_all6(P, d_r, d_i1, d_i2, ws, s);
    Exec X(P, s);
    X.single(ws);
    X.zflags = X.comb_flags(ws);
    X.zflags_n = X.comb_flag_words(P, P.total);
    X.defer_double = true;   // itft + scale back to back
    X.fold = P.fold != 0;    // f4: no scaling pass, the combine reads the reduced form
    X.fuse_row_last = true;  // last row level inside the pointwise (nested negacyclic sizes)
    ProfCall pc;
    int rc;
    pc.mark(0, s);
    if (hb && hb->h) {   // operand 1's forward transform overlaps operand 2's H2D copy
        // kernels first: a copy from pageable memory may hold the calling thread until it is done
        if ((rc = X.fwd_columns(d_i1, P.n1, d_i2, P.n2, 1, 0))) return rc;
        if ((rc = X.fwd_rows(1, 0))) return rc;
        HIPCHK(hipMemcpyAsync((void *)d_i2, hb->h, (size_t)P.n2 * 8, hipMemcpyHostToDevice, hb->cs));
        HIPCHK(hipEventRecord(hb->ready, hb->cs));
        HIPCHK(hipStreamWaitEvent(s, hb->ready, 0));
        if ((rc = X.fwd_columns(d_i1, P.n1, d_i2, P.n2, 1, 1))) return rc;
        if ((rc = X.fwd_rows(1, 1))) return rc;
        pc.mark(1, s);
    } else {
        if ((rc = X.fwd_columns(d_i1, P.n1, d_i2, P.n2, 2))) return rc;
        pc.mark(1, s);
        if ((rc = X.fwd_rows(2))) return rc;
    }
    pc.mark(2, s);
    if ((rc = X.pointwise())) return rc;
    pc.mark(3, s);
    if ((rc = X.inv_rows())) return rc;
    pc.mark(4, s);
    if ((rc = X.itft(0, P.NR, P.Tr))) return rc;
    pc.mark(5, s);
    if ((rc = X.scale())) return rc;
    pc.mark(6, s);
    rc = X.fold ? X.combine_fold(d_r, ws, X.dbl_lo, X.dbl_hi) : X.combine_single(d_r, ws);
    pc.mark(7, s);
    return rc;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

// Which kernel carries each stage for these parameters (the same decisions Exec makes).
int mpfft_stage_kernels(long n1, long n2, unsigned long depth, unsigned long w, char *buf, size_t len)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    const char *pass = P.big ? (P.rpass ? "k_rpass" : "k_bpass") : (P.wave && P.lds) ? "k_lpass" : P.wave ? "k_wpass" : "k_pass";
    char pw[96];
    const int lk = Exec::pwss_lk(P.l);
    const char *rows = P.big && P.rpass && !(lk && pw_get(pw_inner_limbs(P.l, lk), lk)) ? "k_rpass + k_bpass (canonical last pass)" : pass;
    const char *fz = diag_env("MPFFT_FUSE_ROW");
    const bool fused = P.has_c && !(fz && !strcmp(fz, "0"));   // as Exec::row_fused() in run_all
    if (lk && pw_get(pw_inner_limbs(P.l, lk), lk))
        snprintf(pw, sizeof pw, "k_pwss<%d>%s (nested negacyclic, K=%d)", pw_inner_limbs(P.l, lk),
                 !fused ? "" : P.fuse_rows == 2 ? " quad + last two row levels" : " pair + last row level", 1 << lk);
    else if (P.l % 256 == 0 && P.l <= 4096 && pw_kind() != PW_MFMA1 && pw_kind() != PW_VALU)
        snprintf(pw, sizeof pw, "k_pwm2 (int8 MFMA)");
    else if (P.l % 128 == 0 && pw_kind() != PW_VALU)
        snprintf(pw, sizeof pw, "k_pwm (int8 MFMA)");
    else if (P.l % 2 == 0 && P.l >= 32)
        snprintf(pw, sizeof pw, "k_pw (VALU)");
    else
        snprintf(pw, sizeof pw, "k_pointwise (VALU)");
    const char *pair = P.rpass ? "k_rpair" : P.wave ? "k_wpair" : "k_pairop";
    const char *scale = P.fuse_scale ? "(fused into the last inverse column pass)"
                        : P.fold ? "(folded: 2^-(depth+1) in the last inverse row pass)"
                        : P.rpass ? "k_rscale" : P.wave ? "k_wscale" : "k_scale";
    const char *comb = P.fold ? "k_cmeta + k_combine_red (reduced form)" : "k_combine1";
    snprintf(buf, len, "%s;%s;%s;%s;%s + %s;%s;%s", pass, rows, pw, pass, pass, pair, scale, comb);
    return MPFFT_OK;
}

int mpfft_profile_begin(int max_calls)
{
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (max_calls < 1 || g_prof.inflight > 0) return MPFFT_EINVAL;
    const int per = MPFFT_NSTAGES + 1;
    if (g_prof.cap < max_calls) {
        for (int i = 0; i < g_prof.cap * per; ++i) (void)hipEventDestroy(g_prof.ev[i]);
        free(g_prof.ev);
        free(g_prof.marks);
        g_prof.cap = 0;
        g_prof.ev = (hipEvent_t *)calloc((size_t)max_calls * per, sizeof(hipEvent_t));
        g_prof.marks = (int *)calloc((size_t)max_calls, sizeof(int));
        if (!g_prof.ev || !g_prof.marks) return MPFFT_ENOMEM;
        for (int i = 0; i < max_calls * per; ++i)
            if (hipEventCreate(&g_prof.ev[i]) != hipSuccess) {   // no leak: destroy what was made
                for (int j = 0; j < i; ++j) (void)hipEventDestroy(g_prof.ev[j]);
                return MPFFT_EHIP;
            }
        g_prof.cap = max_calls;
    }
    for (int c = 0; c < g_prof.cap; ++c) g_prof.marks[c] = 0;
    g_prof.used = 0;
    g_prof.on = true;
    return MPFFT_OK;
}

// sums the calls that recorded every stage boundary (a call that failed part-way is skipped)
int mpfft_profile_end(float *stage_ms, int *calls)
{
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof.on = false;
    for (int k = 0; k < MPFFT_NSTAGES; ++k) stage_ms[k] = 0.f;
    int done = 0;
    for (int c = 0; c < g_prof.used; ++c) {
        if (g_prof.marks[c] != MPFFT_NSTAGES + 1) continue;
        hipEvent_t *e = g_prof.ev + (size_t)c * (MPFFT_NSTAGES + 1);
        if (hipEventSynchronize(e[MPFFT_NSTAGES]) != hipSuccess) return MPFFT_EHIP;
        for (int k = 0; k < MPFFT_NSTAGES; ++k) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, e[k], e[k + 1]) != hipSuccess) return MPFFT_EHIP;
            stage_ms[k] += ms;
        }
        ++done;
    }
    if (calls) *calls = done;
    return MPFFT_OK;
}

const char *mpfft_strerror(int code)
{
    switch (code) {
    case MPFFT_OK: return "ok";
    case MPFFT_EINVAL: return "invalid parameters (need n1,n2 >= 1, 2 <= depth <= 30, n*w % 64 == 0)";
    case MPFFT_ETOOBIG: return "operands too large for the convolution: need j1 + j2 - 1 <= 2^(depth+1)";
    case MPFFT_EUNSUPPORTED: return "coefficient size n*w/64 > 4096 limbs is not supported";
    case MPFFT_ENOMEM: return "device allocation failed";
    case MPFFT_EHIP: return hipGetErrorString(last_hip_error);
    case MPFFT_ENODEV: return "no HIP device";
    }
    return "unknown error";
}

int mpfft_version(void) { return MPFFT_VERSION; }

int mpfft_check_params(long n1, long n2, unsigned long depth, unsigned long w)
{
    Plan P;
    return make_plan(&P, n1, n2, depth, w);
}

size_t mpfft_workspace_bytes(long n1, long n2, unsigned long depth, unsigned long w)
{
    Plan P;
    if (make_plan(&P, n1, n2, depth, w)) return 0;
    return P.bytes;
}

int mpfft_workspace_layout(long n1, long n2, unsigned long depth, unsigned long w, size_t *out)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    out[0] = P.off_digA; out[1] = P.off_topA; out[2] = P.off_cbA;
    out[3] = P.off_digB; out[4] = P.off_topB; out[5] = P.off_cbB;
    out[6] = P.slots; out[7] = (size_t)cb_words((int)P.l);
    return MPFFT_OK;
}

int mpfft_plan_info(long n1, long n2, unsigned long depth, unsigned long w, long *out)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    out[0] = P.n; out[1] = P.l; out[2] = P.NC; out[3] = P.j1; out[4] = P.j2;
    out[5] = P.trunc; out[6] = (long)P.bits1; out[7] = P.NR; out[8] = P.tpb; out[9] = P.U;
    return MPFFT_OK;
}

int mpfft_mul_device(uint64_t *d_r, const uint64_t *d_i1, long n1, const uint64_t *d_i2, long n2,
                     unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    if (!d_ws || ws_bytes < P.bytes) return MPFFT_ENOMEM;
    (void)hipGetLastError();  // clear a sticky error left by another library in this process
    return run_all(P, d_r, d_i1, d_i2, (unsigned char *)d_ws, (hipStream_t)stream);
}

// stage entry points (device pointers), used by the stage-parity tests and the
// multi-GPU driver.  `ws` has the single-GPU workspace layout for (n1, n2, depth, w).
int mpfft_stage(int stage, const uint64_t *d_i1, const uint64_t *d_i2, uint64_t *d_r, long n1, long n2,
                unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    if (!d_ws || ws_bytes < P.bytes) return MPFFT_ENOMEM;
    (void)hipGetLastError();
    Exec X(P, (hipStream_t)stream);
    X.single((unsigned char *)d_ws);
    switch (stage) {
    case MPFFT_STAGE_FWD_COLUMNS: return X.fwd_columns(d_i1, n1, d_i2, n2, 2);
    case MPFFT_STAGE_FWD_ROWS: return X.fwd_rows(2);
    case MPFFT_STAGE_POINTWISE: return X.pointwise();
    case MPFFT_STAGE_INV_ROWS: return X.inv_rows();
    case MPFFT_STAGE_INV_COLUMNS: return X.itft(0, P.NR, P.Tr);
    case MPFFT_STAGE_SCALE: return X.scale();
    case MPFFT_STAGE_COMBINE: return X.combine_single(d_r, (unsigned char *)d_ws);
    case MPFFT_STAGE_FOLD_COMBINE: {
        if (!P.fold) return MPFFT_EUNSUPPORTED;
        long lo, hi;
        plan_dbl(P, &lo, &hi);
        return X.combine_fold(d_r, (unsigned char *)d_ws, lo, hi);
    }
    }
    return MPFFT_EINVAL;
}

// ---- sharded multi-GPU stages ------------------------------------------------
static int shard_exec(Exec &X, const mpfft_shard *sh)
{
    const Plan &P = X.P;
    if (sh->ccount < 1 || sh->c0 < 0 || sh->c0 + sh->ccount > P.NC) return MPFFT_EINVAL;
    if (sh->rcount < 0 || sh->r0 < 0 || sh->r0 + sh->rcount > P.Tr) return MPFFT_EINVAL;
    if (sh->ccb < 1 || P.NC % sh->ccb || (sh->ccb & (sh->ccb - 1))) return MPFFT_EINVAL;
    for (int k = 0; k < 2; ++k) {
        X.col.dig[k] = sh->col_dig[k];
        X.col.cb[k] = sh->col_cb[k];
        X.col.top[k] = sh->col_top[k];
        X.row.dig[k] = sh->row_dig[k];
        X.row.cb[k] = sh->row_cb[k];
        X.row.top[k] = sh->row_top[k];
    }
    X.c0 = sh->c0;
    X.ccount = sh->ccount;
    X.r0 = sh->r0;
    X.rcount = sh->rcount;
    X.ccb = sh->ccb;
    X.cbb = ilog2(sh->ccb);
    X.cbs = (long)sh->rcount * sh->ccb;
    X.src_chunk = sh->src_chunk;
    if (sh->rowc_dig && sh->rowc_cb && sh->rowc_top) {   // fused last row level (mpfft_shard_row_fused)
        X.cview.dig[0] = sh->rowc_dig;
        X.cview.cb[0] = sh->rowc_cb;
        X.cview.top[0] = sh->rowc_top;
        X.fuse_row_last = true;
    }
    return MPFFT_OK;
}

// The row stages on local rows [lo, hi) only (a row chunk: its exchange #2 can start while the
// next chunk computes).  The row layout keeps its block stride (rcount ccb slots per column
// block); the row passes take the chunk through their row offset and count, the pointwise is
// launched once per column block on the chunk's contiguous slots.
int mpfft_shard_stage_rows(int stage, const mpfft_shard *sh, int lo, int hi, void *stream)
{
    Plan P;
    int rc = make_plan(&P, sh->n1, sh->n2, sh->depth, sh->w);
    if (rc) return rc;
    if (lo < 0 || hi > sh->rcount || lo > hi) return MPFFT_EINVAL;
    if (stage != MPFFT_SHARD_FWD_ROWS && stage != MPFFT_SHARD_POINTWISE && stage != MPFFT_SHARD_INV_ROWS)
        return MPFFT_EINVAL;
    if (lo == hi) return MPFFT_OK;
    (void)hipGetLastError();
    Exec X(P, (hipStream_t)stream);
    if ((rc = shard_exec(X, sh))) return rc;
    const long cbw = cb_words((int)P.l);
    auto shift = [&](View &v, long slots, int nk) {
        for (int k = 0; k < nk; ++k)
            if (v.dig[k]) {
                v.dig[k] += slots * P.l;
                v.cb[k] += slots * cbw;
                v.top[k] += slots;
            }
    };
    // X.cbs (the block stride) stays the full rcount ccb
    shift(X.row, (long)lo * X.ccb, 2);
    shift(X.cview, (long)lo * X.ccb, 1);
    X.r0 += lo;
    X.rcount = hi - lo;
    if (stage == MPFFT_SHARD_FWD_ROWS) return X.fwd_rows(2);
    if (stage == MPFFT_SHARD_INV_ROWS) return X.inv_rows();
    for (long b = 0; b < P.NC / X.ccb; ++b) {   // the pointwise: one launch per column block
        Exec Y = X;
        shift(Y.row, b * X.cbs, 2);
        shift(Y.cview, b * X.cbs, 1);
        Y.pw_count = (long)(hi - lo) * X.ccb;
        if ((rc = Y.pointwise())) return rc;
    }
    return MPFFT_OK;
}

int mpfft_shard_row_fused(long n1, long n2, unsigned long depth, unsigned long w, int ccb)
{
    Plan P;
    if (make_plan(&P, n1, n2, depth, w)) return 0;
    return P.has_c && pw_pair_kernel(P.l, P.fuse_rows) && ccb >= (1 << P.fuse_rows) && !(P.NC % ccb);
}

int mpfft_shard_stage(int stage, const mpfft_shard *sh, const uint64_t *d_i1, const uint64_t *d_i2, void *stream)
{
    Plan P;
    int rc = make_plan(&P, sh->n1, sh->n2, sh->depth, sh->w);
    if (rc) return rc;
    (void)hipGetLastError();
    Exec X(P, (hipStream_t)stream);
    if ((rc = shard_exec(X, sh))) return rc;
    switch (stage) {
    case MPFFT_SHARD_FWD_COLUMNS: return X.fwd_columns(d_i1, sh->n1, d_i2, sh->n2, 2);
    case MPFFT_SHARD_FWD_COLUMNS_A: return X.fwd_columns(d_i1, sh->n1, d_i2, sh->n2, 2, 0);
    case MPFFT_SHARD_FWD_COLUMNS_B: return X.fwd_columns(d_i1, sh->n1, d_i2, sh->n2, 2, 1);
    case MPFFT_SHARD_FWD_COLUMNS_OWN:
        X.own_lo = sh->r0;
        X.own_hi = sh->r0 + sh->rcount;
        return X.fwd_columns(d_i1, sh->n1, d_i2, sh->n2, 2);
    case MPFFT_SHARD_FWD_ROWS: return X.rcount ? X.fwd_rows(2) : MPFFT_OK;
    case MPFFT_SHARD_POINTWISE: return X.pointwise();
    case MPFFT_SHARD_INV_ROWS: return X.rcount ? X.inv_rows() : MPFFT_OK;
    case MPFFT_SHARD_INV_COLUMNS:
        X.defer_double = true;
        if ((rc = X.itft(0, P.NR, P.Tr))) return rc;
        return X.scale();
    }
    return MPFFT_EINVAL;
}

// the stripes of one rank of the column-sharded multiply (multi.hip mpfft_shard_partition):
// stripe j of rank g (g = c0 / ccount of G = NC / ccount ranks) is product stripe j G + g,
// coefficients [(j G + g) C, + C) = column-layout row j of the rank
static void shard_comb_args(const Plan &P, const mpfft_shard *sh, CombArgs *a, long *nst, long *stripe_limbs)
{
    memset(a, 0, sizeof(*a));
    a->C = sh->ccount;
    a->G = (int)(P.NC / sh->ccount);
    a->g = sh->c0 / sh->ccount;
    a->S = (long)a->G * P.Tr;
    *nst = P.Tr;
    // limbs of a stripe at most: ms(s+1) - ms(s) <= ceil(C bits1 / 64); the last stripe runs to
    // the product's end, 64 total <= (len + 1) bits1 <= (T + 1) bits1: at most (C + 1) bits1 / 64 + 2
    *stripe_limbs = (long)((((u64)sh->ccount + 1) * P.bits1) / 64) + 2;
}

size_t mpfft_shard_combine_tmp_bytes(long n1, long n2, unsigned long depth, unsigned long w, int world)
{
    Plan P;
    if (make_plan(&P, n1, n2, depth, w) || world < 1 || P.NC % world) return 0;
    const long sl = (long)((((u64)(P.NC / world) + 1) * P.bits1) / 64) + 2;
    const long nb = P.Tr * Exec::comb_blocks(P, sl);
    return align_up((size_t)(nb + 1) * 4, 256) + align_up((size_t)nb * 4, 256);
}

int mpfft_shard_combine(const mpfft_shard *sh, int phase, uint64_t *d_r, const uint64_t *d_halo, int *d_sums,
                        const int *d_sums_all, void *d_tmp, size_t tmp_bytes, void *stream)
{
    Plan P;
    int rc = make_plan(&P, sh->n1, sh->n2, sh->depth, sh->w);
    if (rc) return rc;
    if (sh->ccount < 1 || P.NC % sh->ccount || sh->c0 % sh->ccount) return MPFFT_EINVAL;
    const int world = (int)(P.NC / sh->ccount);
    if (tmp_bytes < mpfft_shard_combine_tmp_bytes(sh->n1, sh->n2, sh->depth, sh->w, world)) return MPFFT_ENOMEM;
    const long H = (long)((P.N + 128 + P.bits1 - 1) / P.bits1) + 1;
    if (phase == 0 && (!d_sums || (!d_halo && (long)world * P.Tr > 1))) return MPFFT_EINVAL;
    if (phase == 1 && !d_sums_all) return MPFFT_EINVAL;
    (void)hipGetLastError();
    Exec X(P, (hipStream_t)stream);
    if ((rc = shard_exec(X, sh))) return rc;
    CombArgs a;
    long nst, sl;
    shard_comb_args(P, sh, &a, &nst, &sl);
    a.dig = X.col.dig[0];
    a.halo = d_halo;
    a.H = (int)H;
    a.SL = sl;
    const long nb = nst * Exec::comb_blocks(P, sl);
    u32 *st = (u32 *)d_tmp;
    u32 *allp = (u32 *)((unsigned char *)d_tmp + align_up((size_t)(nb + 1) * 4, 256));
    hipStream_t s = (hipStream_t)stream;
    if (phase == 0) {   // every stripe with carry-in 0, and its (generate, propagate) summary
        if ((rc = X.combine1(a, nst, sl, d_r, st, false, allp))) return rc;
        hipLaunchKernelGGL(k_comb_summary, dim3((unsigned)nst), dim3(256), 0, s, (const u32 *)st, (const u32 *)allp,
                           Exec::comb_blocks(P, sl), d_sums);
        HIPCHK(hipGetLastError());
        return MPFFT_OK;
    }
    // the carries between stripes, from every rank's summaries
    a.l = (int)P.l;
    a.N = P.N;
    a.bits1 = P.bits1;
    a.len = P.len;
    a.total = P.total;
    hipLaunchKernelGGL(k_stripe_carry, dim3((unsigned)nst), dim3(256), 0, s, a, nst, d_sums_all, d_r);
    HIPCHK(hipGetLastError());
    return MPFFT_OK;
}

// host-pointer entry with status.  One context per device (SURVEY 8b "Threading"):
// the calling thread's current HIP device selects it, so threads driving different
// GPUs never share memory or streams; threads on the same device serialise on its lock.
struct DevCtx {
    std::mutex mu;
    unsigned char *ws = nullptr;
    size_t ws_bytes = 0;
    u64 *io = nullptr;
    size_t io_bytes = 0;
    hipStream_t stream = nullptr;
    hipStream_t copy = nullptr;   // operand 2's H2D beside operand 1's forward transform
    hipEvent_t ready = nullptr;
};
static const int MPFFT_MAX_DEV = 64;
static DevCtx g_dev[MPFFT_MAX_DEV];

// grow-only device buffer owned by a DevCtx
static int ensure_buf(void **p, size_t *have, size_t need)
{
    if (*have >= need) return MPFFT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipMalloc(p, need) != hipSuccess) return MPFFT_ENOMEM;
    *have = need;
    return MPFFT_OK;
}

static int mul_host(const Plan &P, uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2)
{
    int rc;
    (void)hipGetLastError();
    int ndev = 0, dev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MPFFT_ENODEV;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MPFFT_MAX_DEV) return MPFFT_ENODEV;
    DevCtx &C = g_dev[dev];
    std::lock_guard<std::mutex> lk(C.mu);
    if (!C.stream) HIPCHK(hipStreamCreateWithFlags(&C.stream, hipStreamNonBlocking));
    if (!C.copy) HIPCHK(hipStreamCreateWithFlags(&C.copy, hipStreamNonBlocking));
    if (!C.ready) HIPCHK(hipEventCreateWithFlags(&C.ready, hipEventDisableTiming));
    if ((rc = ensure_buf((void **)&C.ws, &C.ws_bytes, P.bytes))) return rc;
    if ((rc = ensure_buf((void **)&C.io, &C.io_bytes, (size_t)2 * (n1 + n2) * 8))) return rc;
    u64 *d_i1 = C.io, *d_i2 = C.io + n1, *d_r = C.io + n1 + n2;
    HIPCHK(hipMemcpyAsync(d_i1, i1, (size_t)n1 * 8, hipMemcpyHostToDevice, C.stream));
    HostB hb{P.sqrt2 ? nullptr : i2, C.copy, C.ready};
    if (P.sqrt2) HIPCHK(hipMemcpyAsync(d_i2, i2, (size_t)n2 * 8, hipMemcpyHostToDevice, C.stream));
    rc = run_all(P, d_r, d_i1, d_i2, C.ws, C.stream, &hb);
    if (rc) {
        (void)hipStreamSynchronize(C.copy);   // the copy stream never outlives the call
        return rc;
    }
    HIPCHK(hipMemcpyAsync(r1, d_r, (size_t)(n1 + n2) * 8, hipMemcpyDeviceToHost, C.stream));
    HIPCHK(hipStreamSynchronize(C.stream));
    return MPFFT_OK;
}

static thread_local int g_last_ngpus = 0;
int mpfft_last_ngpus(void) { return g_last_ngpus; }

int mpfft_mul_ex(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2, unsigned long depth,
                 unsigned long w)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w);
    if (rc) return rc;
    std::vector<int> devs;
    if (mpfft_multi_policy(n1, n2, depth, w, devs) > 1) {   // column-sharded over the policy's devices
        g_last_ngpus = (int)devs.size();
        rc = mpfft_mul_multi(r1, i1, n1, i2, n2, depth, w, (int)devs.size(), devs.data());
        // the policy's devices missing or full: the product still fits one device
        if (rc != MPFFT_ENODEV && rc != MPFFT_ENOMEM) return rc;
    }
    g_last_ngpus = 1;
    return mul_host(P, r1, i1, n1, i2, n2);
}

// ---- the sqrt2 front end new_mpn_mul6 (mul_fft.c:3573-3668) ---------
int mpfft_check_params6(long n1, long n2, unsigned long depth, unsigned long w)
{
    Plan P;
    return make_plan(&P, n1, n2, depth, w, true);
}

size_t mpfft_workspace_bytes6(long n1, long n2, unsigned long depth, unsigned long w)
{
    Plan P;
    if (make_plan(&P, n1, n2, depth, w, true)) return 0;
    return P.bytes;
}

int mpfft_plan_info6(long n1, long n2, unsigned long depth, unsigned long w, long *out)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w, true);
    if (rc) return rc;
    out[0] = P.n; out[1] = P.l; out[2] = P.NC; out[3] = P.j1; out[4] = P.j2;
    out[5] = P.trunc; out[6] = (long)P.bits1; out[7] = P.NR; out[8] = P.tpb; out[9] = P.U;
    return MPFFT_OK;
}

int mpfft_mul6_device(uint64_t *d_r, const uint64_t *d_i1, long n1, const uint64_t *d_i2, long n2,
                      unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w, true);
    if (rc) return rc;
    if (!d_ws || ws_bytes < P.bytes) return MPFFT_ENOMEM;
    (void)hipGetLastError();
    return run_all(P, d_r, d_i1, d_i2, (unsigned char *)d_ws, (hipStream_t)stream);
}

int mpfft_mul6_ex(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2, unsigned long depth,
                  unsigned long w)
{
    Plan P;
    int rc = make_plan(&P, n1, n2, depth, w, true);
    if (rc) return rc;
    return mul_host(P, r1, i1, n1, i2, n2);
}

// mul_fft.c:3573 -- same signature and meaning; fails loudly instead of segfaulting
void new_mpn_mul6(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1, mp_limb_t *i2, mp_size_t n2, mp_bitcnt_t depth,
                  mp_bitcnt_t w)
{
    int rc = mpfft_mul6_ex(r1, i1, n1, i2, n2, depth, w);
    if (rc) {
        fprintf(stderr, "new_mpn_mul6(n1=%ld, n2=%ld, depth=%lu, w=%lu): %s\n", (long)n1, (long)n2,
                (unsigned long)depth, (unsigned long)w, mpfft_strerror(rc));
        abort();
    }
}

// release the calling device's cached workspace (the next call re-allocates)
int mpfft_release(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MPFFT_MAX_DEV) return MPFFT_ENODEV;
    DevCtx &C = g_dev[dev];
    std::lock_guard<std::mutex> lk(C.mu);
    if (C.ws) (void)hipFree(C.ws);
    if (C.io) (void)hipFree(C.io);
    C.ws = nullptr;
    C.io = nullptr;
    C.ws_bytes = C.io_bytes = 0;
    return MPFFT_OK;
}

// ---- (depth, w) chooser -------------------------------------------
// The reference leaves (depth, w) to its caller (mul_fft.c:3190-3191); an MPIR-style
// mpn_mul drop-in needs them picked from the operand sizes.  Candidates: every depth in
// [2, 24] and power-of-two w with a whole number of limbs per coefficient, l <= 4096, and
// room for the product (make_plan).  Predicted device time = launches x a launch cost +
// live slots (T) x the measured per-slot cost of a multiply at that coefficient size
// (CHOOSE_SLOT_NS[log2 l], from scripts/chooser_sweep.py on MI355X:
// profiles/r02/chooser_sweep.json); the cheapest candidate wins.  The round-5 re-sweep
// (profiles/r05/chooser_sweep.json: l = 2048 196 ns, l = 4096 512 ns per slot, measured at
// T = 32768 / 16384 slots) is not taken over: a linear per-slot model with those costs picks
// l = 2048 for 10^6-limb products, whose 2048 live slots fill a quarter of the GPU's
// pointwise workgroup slots -- the measured per-slot cost does not hold there.  With the r02
// table the chosen candidate is the fastest of every one timed at all four test sizes
// (profiles/r05/chooser_check.log, tests/test_gpu_chooser.py at 1.2x).  Model: a fixed cost
// (launches: ~0.045 ms for the small configurations of the sweep) + T x the marginal
// per-slot cost at that coefficient size, (ms - 0.045) / T of the sweep.
static const double CHOOSE_SLOT_NS[13] = {69.7, 26.6, 12.3, 10.4, 7.3, 6.6, 11.0, 13.2, 28.4, 98.2, 167.9, 270.0, 810.7};
static const double CHOOSE_FIXED_MS = 0.045;

static double choose_cost(const Plan &P)
{
    const int k = ilog2(P.l);
    return CHOOSE_FIXED_MS + (double)P.trunc * CHOOSE_SLOT_NS[k < 12 ? k : 12] * 1e-6;
}

int mpfft_choose(long n1, long n2, unsigned long *depth, unsigned long *w)
{
    double best = -1.0;
    for (unsigned long d = 2; d <= 24; ++d)
        for (unsigned long wv = 1; wv <= 4096; wv *= 2) {
            const unsigned long long N = (1ull << d) * wv;
            if (N % 64) continue;
            if (N / 64 > 4096) break;
            Plan P;
            if (make_plan(&P, n1, n2, d, wv)) continue;
            const double c = choose_cost(P);
            if (best < 0 || c < best) {
                best = c;
                *depth = d;
                *w = wv;
            }
        }
    return best < 0 ? MPFFT_ETOOBIG : MPFFT_OK;
}

int mpfft_mul_auto(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2)
{
    unsigned long d = 0, wv = 0;
    const int rc = mpfft_choose(n1, n2, &d, &wv);
    if (rc) return rc;
    return mpfft_mul_ex(r1, i1, n1, i2, n2, d, wv);
}

// mul_fft.c:3190 -- same signature and meaning; fails loudly instead of segfaulting
void new_mpn_mul(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1, mp_limb_t *i2, mp_size_t n2, mp_bitcnt_t depth,
                 mp_bitcnt_t w)
{
    int rc = mpfft_mul_ex(r1, i1, n1, i2, n2, depth, w);
    if (rc) {
        fprintf(stderr, "new_mpn_mul(n1=%ld, n2=%ld, depth=%lu, w=%lu): %s\n", (long)n1, (long)n2,
                (unsigned long)depth, (unsigned long)w, mpfft_strerror(rc));
        abort();
    }
}

// splitmix64-seeded xoshiro256** (BASELINE.md synthetic inputs; same stream as the oracle's)
void mpfft_fill_random(uint64_t *buf, long cnt, uint64_t seed)
{
    uint64_t s[4], z = seed;
    for (int i = 0; i < 4; i++) {
        z += 0x9e3779b97f4a7c15ULL;
        uint64_t x = z;
        x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
        x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
        s[i] = x ^ (x >> 31);
    }
    for (long i = 0; i < cnt; i++) {
        const uint64_t r = s[1] * 5;
        buf[i] = ((r << 7) | (r >> 57)) * 9;
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t;
        s[3] = (s[3] << 45) | (s[3] >> 19);
    }
}

}  // extern "C"
