/*
 * oracle/mpfft_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of wbhart/mpir-fft's `new_mpn_mul` hot path
 * (/root/reference/mul_fft.c:3190-3265) and of every function it reaches
 * (SURVEY.md section 8a, rows a1-a22).  It exists to CHECK the MI355X product
 * (mpir-fft_amd/) and to serve as the `cpu_baseline` leg of bench.py.  It is
 * never linked into, loaded by or called from the product path.
 *
 * Why a restatement and not the reference itself: mul_fft.c includes MPIR's
 * mpir.h / gmp-impl.h / longlong.h (mul_fft.c:36-38), which are not in this
 * image.  Building it would require writing stand-ins for those headers,
 * so the reference is treated as unbuildable here ("Oracle").
 *
 * Parity pinning (tests/test_oracle.py):
 *   - the L1 primitives against exact big-integer references that restate the
 *     reference's own mpz oracles (ref_norm, ref_mul_2expmod, ref_div_2expmod,
 *     ref_lshB_sumdiffmod, ref_sumdiff_rshBmod, mul_fft.c:3699-3760) over the
 *     parameter grids of test_norm / test_mul_2expmod / test_div_2expmod /
 *     test_lshB_sumdiffmod / test_sumdiff_rshBmod (mul_fft.c:3777-4186);
 *   - the transforms by the reference's round-trip properties
 *     (test_fft_ifft :4276, test_fft_truncate :5031, test_fft_ifft_truncate
 *     :4472, test_fft_ifft_mfa_truncate :4938) and by the exact slot-map spec
 *     of SURVEY 8a/a3;
 *   - new_mpn_mul end to end against the exact product (Python int and GMP
 *     mpn_mul, the reference's own integration oracle, mul_fft.c:5542) and
 *     against committed golden vectors (tests/golden/).
 *
 * Deliberate difference from the shipped reference: the pointwise loop uses
 * the row bit-reversal width log2(NR) = depth + 1 - depth/2 instead of
 * (depth + 1)/2 (mul_fft.c:3246), without which the
 * reference returns wrong products.
 *
 * Third-party arithmetic: the pointwise product calls MPIR 2.4.0's
 * mpn_mulmod_2expp1 (mul_fft.c:3119-3123), which is not vendored.  It is
 * restated below (o_mulmod_2expp1) on top of GMP's mpn_mul_n, the same
 * full-product-then-fold algorithm MPIR uses for these sizes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t limb_t;
typedef int64_t slimb_t;

/* GMP (libgmp.so.10) -- used only for the schoolbook/Toom full product inside
 * the pointwise mulmod and as the independent end-to-end checker. */
extern void __gmpn_mul_n(limb_t *rp, const limb_t *ap, const limb_t *bp, long n);
extern limb_t __gmpn_mul(limb_t *rp, const limb_t *ap, long an, const limb_t *bp, long bn);

/* ------------------------------------------------------------------------- */
/* mpn layer: the MPIR 2.4 semantics the reference links  */
/* ------------------------------------------------------------------------- */

static limb_t o_add_n(limb_t *r, const limb_t *a, const limb_t *b, long n)
{
    limb_t cy = 0;
    for (long i = 0; i < n; i++) {
        unsigned __int128 s = (unsigned __int128)a[i] + b[i] + cy;
        r[i] = (limb_t)s;
        cy = (limb_t)(s >> 64);
    }
    return cy;
}

static limb_t o_sub_n(limb_t *r, const limb_t *a, const limb_t *b, long n)
{
    limb_t bw = 0;
    for (long i = 0; i < n; i++) {
        unsigned __int128 d = (unsigned __int128)a[i] - b[i] - bw;
        r[i] = (limb_t)d;
        bw = (limb_t)(d >> 64) & 1;
    }
    return bw;
}

/* in-place r += c over n limbs, early exit once the carry dies */
static limb_t o_incr(limb_t *r, long n, limb_t c)
{
    for (long i = 0; i < n && c; i++) {
        limb_t t = r[i] + c;
        c = t < c;
        r[i] = t;
    }
    return c;
}

/* in-place r -= c over n limbs */
static limb_t o_decr(limb_t *r, long n, limb_t c)
{
    for (long i = 0; i < n && c; i++) {
        limb_t t = r[i];
        r[i] = t - c;
        c = t < c;
    }
    return c;
}

/* r = -a mod B^n; returns 1 iff a != 0 (mpn_neg_n, accepts n == 0) */
static limb_t o_neg_n(limb_t *r, const limb_t *a, long n)
{
    limb_t bw = 0;
    for (long i = 0; i < n; i++) {
        limb_t ai = a[i];
        r[i] = (limb_t)0 - ai - bw;
        bw |= (ai != 0);
    }
    return bw;
}

/* 0 < cnt < 64; returns the bits shifted out of the top limb (low bits) */
static limb_t o_lshift(limb_t *r, const limb_t *a, long n, unsigned cnt)
{
    limb_t out = a[n - 1] >> (64 - cnt);
    for (long i = n - 1; i > 0; i--)
        r[i] = (a[i] << cnt) | (a[i - 1] >> (64 - cnt));
    r[0] = a[0] << cnt;
    return out;
}

/* 0 < cnt < 64; returns the bits shifted out of limb 0, left aligned */
static limb_t o_rshift(limb_t *r, const limb_t *a, long n, unsigned cnt)
{
    limb_t out = a[0] << (64 - cnt);
    for (long i = 0; i < n - 1; i++)
        r[i] = (a[i] >> cnt) | (a[i + 1] << (64 - cnt));
    r[n - 1] = a[n - 1] >> cnt;
    return out;
}

static int o_is_zero(const limb_t *a, long n)
{
    for (long i = 0; i < n; i++)
        if (a[i]) return 0;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* L1: arithmetic modulo p = 2^N + 1, N = 64 l, on (l+1)-limb two's          */
/* complement residues (README:50-58)                                        */
/* ------------------------------------------------------------------------- */

/* mul_fft.h:45-58 mpn_addmod_2expp1_1: r += c for a signed limb c, no reduction */
static void o_addmod_1(limb_t *r, long l, slimb_t c)
{
    if (c >= 0) o_incr(r, l + 1, (limb_t)c);
    else o_decr(r, l + 1, (limb_t)0 - (limb_t)c);
}

/* mul_fft.c:272-294 mpn_normmod_2expp1: canonical residue in [0, 2^N].
 * value = lo + hi*B^l == lo - hi; fold until the top limb is 0, or the value
 * is exactly 2^N (top limb 1, rest 0). */
static void o_normmod(limb_t *t, long l)
{
    slimb_t hi = (slimb_t)t[l];
    if (!hi) return;
    t[l] = 0;
    o_addmod_1(t, l, -hi);
    hi = (slimb_t)t[l];              /* now in {-1, 0, 1} */
    if (!hi) return;
    t[l] = 0;
    o_addmod_1(t, l, -hi);
    if (t[l] == ~(limb_t)0) {        /* lo was 0 and hi 1: -1 == 2^N */
        t[l] = 0;
        o_addmod_1(t, l, 1);
    }
}

/* mul_fft.c:470-488 mpn_mul_2expmod_2expp1: t = a * 2^d mod p, 0 <= d < 64 */
static void o_mul_2expmod(limb_t *t, const limb_t *a, long l, unsigned d)
{
    if (!d) {
        if (t != a) memcpy(t, a, (l + 1) * sizeof(limb_t));
        return;
    }
    slimb_t top = (slimb_t)a[l];
    o_lshift(t, a, l + 1, d);
    limb_t h = t[l];                 /* h * B^l == -h */
    t[l] = 0;
    o_decr(t, l + 1, h);
    /* the signed bits pushed out of the top limb weigh B^(l+1) == -B */
    o_addmod_1(t + 1, l - 1, -(top >> (64 - d)));
}

/* mul_fft.c:494-512 mpn_div_2expmod_2expp1: t = a / 2^d mod p, 0 <= d < 64 */
static void o_div_2expmod(limb_t *t, const limb_t *a, long l, unsigned d)
{
    if (!d) {
        if (t != a) memcpy(t, a, (l + 1) * sizeof(limb_t));
        return;
    }
    slimb_t top = (slimb_t)a[l];
    limb_t out = o_rshift(t, a, l + 1, d);
    t[l] = (limb_t)(top >> d);
    /* the d low bits r of a contribute r * 2^-d == -r * 2^(N-d) = -out * B^(l-1) */
    limb_t x = t[l - 1];
    t[l - 1] = x - out;
    t[l] -= (x < out);
}

/* mul_fft.c:926-957 FFT_twiddle generalised to any exponent: r = a * 2^e mod p,
 * 0 <= e < 2N (e >= N carries the sign 2^N == -1).  r must not alias a. */
static void o_mul_2exp(limb_t *r, const limb_t *a, long l, unsigned long e)
{
    unsigned long N = 64UL * (unsigned long)l;
    int neg = 0;
    e %= 2 * N;
    if (e >= N) { neg = 1; e -= N; }
    long x = (long)(e / 64);
    unsigned b = (unsigned)(e % 64);
    if (x) {
        /* a * B^x: limbs [x, l) <- a[0, l-x); the wrapped high limbs come back negated */
        memcpy(r + x, a, (size_t)(l - x) * sizeof(limb_t));
        r[l] = 0;
        limb_t bw = o_neg_n(r, a + l - x, x);
        o_addmod_1(r + x, l - x, -(slimb_t)a[l]);
        o_decr(r + x, l - x + 1, bw);
    } else {
        memcpy(r, a, (size_t)(l + 1) * sizeof(limb_t));
    }
    if (neg) o_neg_n(r, r, l + 1);
    o_mul_2expmod(r, r, l, b);
}

/* ------------------------------------------------------------------------- */
/* L2: butterflies (mul_fft.c:514-752).  Each writes its two outputs into    */
/* the context temporaries and swaps them into the coefficient table, as the */
/* reference does with its t1/t2 pointers.                                   */
/* ------------------------------------------------------------------------- */

typedef struct {
    long l;          /* limbs per coefficient (without the carry limb) */
    unsigned long N; /* 64 l */
    limb_t *t1, *t2, *t3;
} octx;

#define SWAP_PTR(a, b) do { limb_t *s_ = (a); (a) = (b); (b) = s_; } while (0)

/* mul_fft.c:553-576 FFT_radix2_butterfly: s = a + b, t = 2^e (a - b) */
static void o_bfly(octx *c, limb_t **pa, limb_t **pb, unsigned long e)
{
    long l = c->l;
    o_add_n(c->t1, *pa, *pb, l + 1);
    o_sub_n(c->t3, *pa, *pb, l + 1);
    o_mul_2exp(c->t2, c->t3, l, e);
    SWAP_PTR(*pa, c->t1);
    SWAP_PTR(*pb, c->t2);
}

/* mul_fft.c:639-652 FFT_radix2_inverse_butterfly: s = a + 2^-e b, t = a - 2^-e b */
static void o_ibfly(octx *c, limb_t **pa, limb_t **pb, unsigned long e)
{
    long l = c->l;
    o_mul_2exp(c->t3, *pb, l, (2 * c->N - e % (2 * c->N)) % (2 * c->N));
    o_add_n(c->t1, *pa, c->t3, l + 1);
    o_sub_n(c->t2, *pa, c->t3, l + 1);
    SWAP_PTR(*pa, c->t1);
    SWAP_PTR(*pb, c->t2);
}

/* mul_fft.c:517-548 FFT_radix2_twiddle_butterfly: u = 2^b1 (s + t), v = 2^b2 (s - t) */
static void o_tw_bfly(octx *c, limb_t **pa, limb_t **pb, unsigned long b1, unsigned long b2)
{
    long l = c->l;
    o_add_n(c->t3, *pa, *pb, l + 1);
    o_mul_2exp(c->t1, c->t3, l, b1);
    o_sub_n(c->t3, *pa, *pb, l + 1);
    o_mul_2exp(c->t2, c->t3, l, b2);
    SWAP_PTR(*pa, c->t1);
    SWAP_PTR(*pb, c->t2);
}

/* mul_fft.c:721-752 FFT_radix2_twiddle_inverse_butterfly:
 * s = 2^-b1 a + 2^-b2 b, t = 2^-b1 a - 2^-b2 b */
static void o_tw_ibfly(octx *c, limb_t **pa, limb_t **pb, unsigned long b1, unsigned long b2)
{
    long l = c->l;
    unsigned long M = 2 * c->N;
    o_mul_2exp(c->t1, *pa, l, (M - b1 % M) % M);
    o_mul_2exp(c->t3, *pb, l, (M - b2 % M) % M);
    o_add_n(*pa, c->t1, c->t3, l + 1);
    o_sub_n(*pb, c->t1, c->t3, l + 1);
}

/* ------------------------------------------------------------------------- */
/* L3: radix-2 transforms.  Length 2n, root 2^w, coefficients ii[k*is].     */
/* ------------------------------------------------------------------------- */

/* mul_fft.c:786-827 FFT_radix2 (rr == ii on this path): DIF, bit-reversed out */
static void o_fft(octx *c, limb_t **ii, long is, long n, unsigned long w)
{
    for (long i = 0; i < n; i++)
        o_bfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
    if (n > 1) {
        o_fft(c, ii, is, n / 2, 2 * w);
        o_fft(c, ii + n * is, is, n / 2, 2 * w);
    }
}

/* mul_fft.c:1397-1442 FFT_radix2_twiddle: DIF whose bottom butterflies also apply
 * the MFA twiddles 2^(ws*r*c) and 2^(ws*(r+rs)*c) (README:89) */
static void o_fft_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                     unsigned long ws, long r, long col, long rs)
{
    if (n == 1) {
        unsigned long tw1 = (unsigned long)(r * col), tw2 = tw1 + (unsigned long)(rs * col);
        o_tw_bfly(c, &ii[0], &ii[is], tw1 * ws, tw2 * ws);
        return;
    }
    for (long i = 0; i < n; i++)
        o_bfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
    o_fft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    o_fft_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs);
}

/* mul_fft.c:1076-1122 FFT_radix2_truncate1_twiddle: only outputs < trunc wanted,
 * inputs are all live */
static void o_fft_trunc1_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                            unsigned long ws, long r, long col, long rs, long trunc)
{
    if (trunc == 2 * n) {
        o_fft_tw(c, ii, is, n, w, ws, r, col, rs);
        return;
    }
    if (trunc <= n) {
        /* only the "sum" half is wanted */
        for (long i = 0; i < n; i++)
            o_add_n(ii[i * is], ii[i * is], ii[(i + n) * is], c->l + 1);
        o_fft_trunc1_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs, trunc);
        return;
    }
    for (long i = 0; i < n; i++)
        o_bfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
    o_fft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    o_fft_trunc1_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs, trunc - n);
}

/* mul_fft.c:1179-1228 FFT_radix2_truncate_twiddle: inputs >= trunc are zero and
 * never read, only outputs < trunc are produced (van der Hoeven, README:93-127) */
static void o_fft_trunc_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                           unsigned long ws, long r, long col, long rs, long trunc)
{
    if (trunc == 2 * n) {
        o_fft_tw(c, ii, is, n, w, ws, r, col, rs);
        return;
    }
    if (trunc <= n) {                /* case (a): A 0 0 0 */
        o_fft_trunc_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs, trunc);
        return;
    }
    /* case (b): A A A 0 */
    for (long i = 0; i < trunc - n; i++)
        o_bfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
    for (long i = trunc; i < 2 * n; i++)      /* zero partner: diff = 2^((i-n)w) x */
        o_mul_2exp(ii[i * is], ii[(i - n) * is], c->l, (unsigned long)(i - n) * w);
    o_fft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    o_fft_trunc1_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs, trunc - n);
}

/* mul_fft.c:1444-1486 IFFT_radix2: DIT, bit-reversed in, natural out, result x 2n */
static void o_ifft(octx *c, limb_t **ii, long is, long n, unsigned long w)
{
    if (n > 1) {
        o_ifft(c, ii, is, n / 2, 2 * w);
        o_ifft(c, ii + n * is, is, n / 2, 2 * w);
    }
    for (long i = 0; i < n; i++)
        o_ibfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
}

/* mul_fft.c:1964-2010 IFFT_radix2_twiddle */
static void o_ifft_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                      unsigned long ws, long r, long col, long rs)
{
    if (n == 1) {
        unsigned long tw1 = (unsigned long)(r * col), tw2 = tw1 + (unsigned long)(rs * col);
        o_tw_ibfly(c, &ii[0], &ii[is], tw1 * ws, tw2 * ws);
        return;
    }
    o_ifft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    o_ifft_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs);
    for (long i = 0; i < n; i++)
        o_ibfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
}

/* mul_fft.c:1604-1668 IFFT_radix2_truncate1_twiddle: outputs [0, trunc) known,
 * inputs [trunc, 2n) known (already scaled by 2n) and stored in place */
static void o_ifft_trunc1_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                             unsigned long ws, long r, long col, long rs, long trunc)
{
    long l = c->l;
    if (trunc == 2 * n) {
        o_ifft_tw(c, ii, is, n, w, ws, r, col, rs);
        return;
    }
    if (trunc <= n) {
        for (long i = trunc; i < n; i++) {   /* sub-problem inputs (x_i + x_{i+n}) n */
            o_add_n(ii[i * is], ii[i * is], ii[(i + n) * is], l + 1);
            o_div_2expmod(ii[i * is], ii[i * is], l, 1);
        }
        o_ifft_trunc1_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs, trunc);
        for (long i = 0; i < trunc; i++) {   /* 2n x_i = 2 (n s_i) - 2n x_{i+n} */
            o_add_n(ii[i * is], ii[i * is], ii[i * is], l + 1);
            o_sub_n(ii[i * is], ii[i * is], ii[(n + i) * is], l + 1);
        }
        return;
    }
    o_ifft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    for (long i = trunc - n; i < n; i++) {
        /* d = n s_i - 2n x_{i+n} = n (x_i - x_{i+n}); the right half needs 2^(iw) d,
         * and 2n x_i = n s_i + d */
        o_sub_n(ii[(i + n) * is], ii[i * is], ii[(i + n) * is], l + 1);
        o_mul_2exp(c->t1, ii[(i + n) * is], l, (unsigned long)i * w);
        o_add_n(ii[i * is], ii[i * is], ii[(i + n) * is], l + 1);
        SWAP_PTR(ii[(i + n) * is], c->t1);
    }
    o_ifft_trunc1_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs, trunc - n);
    for (long i = 0; i < trunc - n; i++)
        o_ibfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
}

/* mul_fft.c:1733-1790 IFFT_radix2_truncate_twiddle: outputs [0, trunc) known,
 * inputs >= trunc known to be zero (README:129-189) */
static void o_ifft_trunc_tw(octx *c, limb_t **ii, long is, long n, unsigned long w,
                            unsigned long ws, long r, long col, long rs, long trunc)
{
    long l = c->l;
    if (trunc == 2 * n) {
        o_ifft_tw(c, ii, is, n, w, ws, r, col, rs);
        return;
    }
    if (trunc <= n) {                /* case (a): recurse, then double */
        o_ifft_trunc_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs, trunc);
        for (long i = 0; i < trunc; i++)
            o_add_n(ii[i * is], ii[i * is], ii[i * is], l + 1);
        return;
    }
    /* case (b) */
    o_ifft_tw(c, ii, is, n / 2, 2 * w, ws, r, col, 2 * rs);
    for (long i = trunc; i < 2 * n; i++)     /* x_i = 0 there: d_{i-n} = 2^((i-n)w) s_{i-n} */
        o_mul_2exp(ii[i * is], ii[(i - n) * is], l, (unsigned long)(i - n) * w);
    o_ifft_trunc1_tw(c, ii + n * is, is, n / 2, 2 * w, ws, r + rs, col, 2 * rs, trunc - n);
    for (long i = 0; i < trunc - n; i++)
        o_ibfly(c, &ii[i * is], &ii[(n + i) * is], (unsigned long)i * w);
    for (long i = trunc - n; i < n; i++)
        o_add_n(ii[i * is], ii[i * is], ii[i * is], l + 1);
}

/* ------------------------------------------------------------------------- */
/* L0 + L4: revbin, split/combine, truncated matrix Fourier algorithm        */
/* ------------------------------------------------------------------------- */

/* mul_fft.c:63-79 mpir_revbin (a plain loop for every width; the reference's
 * table path reads out of bounds for in >= 2^bits) */
static long o_revbin(long in, unsigned bits)
{
    long out = 0;
    for (unsigned i = 0; i < bits; i++) {
        out = (out << 1) | (in & 1);
        in >>= 1;
    }
    return out;
}

static unsigned o_log2(long v)
{
    unsigned d = 0;
    while ((1L << d) < v) d++;
    return d;
}

/* bits [start, start + count) of src (nlimbs long; bits past the end read 0) into dst */
static void o_extract_bits(limb_t *dst, const limb_t *src, long nlimbs,
                           unsigned long start, unsigned long count)
{
    long q = (long)(start / 64);
    unsigned sh = (unsigned)(start % 64);
    long words = (long)((count + 63) / 64);
    for (long k = 0; k < words; k++) {
        limb_t lo = (q + k < nlimbs) ? src[q + k] : 0;
        limb_t hi = (sh && q + k + 1 < nlimbs) ? src[q + k + 1] : 0;
        dst[k] = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    }
    unsigned rem = (unsigned)(count % 64);
    if (rem) dst[words - 1] &= (((limb_t)1) << rem) - 1;
}

/* mul_fft.c:115-170 FFT_split_bits (and its limb-aligned special case FFT_split,
 * :87-106): coefficient j = bits [j bits, (j+1) bits) of src, zero padded to l+1
 * limbs; returns the number of coefficients ceil(64 nlimbs / bits) */
static long o_split_bits(limb_t **poly, const limb_t *src, long nlimbs,
                         unsigned long bits, long l)
{
    long len = (long)((64UL * (unsigned long)nlimbs - 1) / bits + 1);
    unsigned long total = 64UL * (unsigned long)nlimbs;
    for (long j = 0; j < len; j++) {
        unsigned long start = (unsigned long)j * bits;
        unsigned long cnt = (start + bits <= total) ? bits : total - start;
        memset(poly[j], 0, (size_t)(l + 1) * sizeof(limb_t));
        o_extract_bits(poly[j], src, nlimbs, start, cnt);
    }
    return len;
}

/* mul_fft.c:207-267 FFT_combine_bits (and FFT_combine, :180-197):
 * res += sum_j poly[j] 2^(j bits), clipped at total limbs; res zeroed by the caller */
static void o_combine_bits(limb_t *res, limb_t **poly, long len, unsigned long bits,
                           long l, long total)
{
    limb_t *tmp = (limb_t *)malloc((size_t)(l + 2) * sizeof(limb_t));
    for (long j = 0; j < len; j++) {
        unsigned long start = (unsigned long)j * bits;
        long off = (long)(start / 64);
        unsigned sh = (unsigned)(start % 64);
        if (off >= total) break;
        tmp[l + 1] = 0;
        memcpy(tmp, poly[j], (size_t)(l + 1) * sizeof(limb_t));
        if (sh) tmp[l + 1] = o_lshift(tmp, tmp, l + 1, sh);
        long cnt = l + 2;
        if (off + cnt > total) cnt = total - off;
        limb_t cy = o_add_n(res + off, res + off, tmp, cnt);
        if (cy && off + cnt < total) o_incr(res + off + cnt, total - off - cnt, cy);
    }
    free(tmp);
}

/* mul_fft.c:2357-2409 FFT_radix2_mfa_truncate.  n2 = 2n/n1 rows of n1 columns.
 * Output spec: slot r*n1 + c = X_{r + n2 c} normalised, for the
 * computed rows r = revbin(s, log2 n2), s < trunc/n1. */
static void o_fft_mfa_trunc(octx *c, limb_t **ii, long n, unsigned long w, long n1, long trunc)
{
    long n2 = 2 * n / n1;
    unsigned dr = o_log2(n2), dc = o_log2(n1);
    long tr = trunc / n1;
    for (long col = 0; col < n1; col++) {
        o_fft_trunc_tw(c, ii + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1, tr);
        for (long j = 0; j < n2; j++) {
            long s = o_revbin(j, dr);
            if (j < s) SWAP_PTR(ii[col + j * n1], ii[col + s * n1]);
        }
    }
    for (long s = 0; s < tr; s++) {
        long row = o_revbin(s, dr);
        limb_t **rp = ii + row * n1;
        o_fft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
        for (long j = 0; j < n1; j++) {
            long t = o_revbin(j, dc);
            if (j < t) SWAP_PTR(rp[j], rp[t]);
        }
        for (long j = 0; j < n1; j++) o_normmod(rp[j], c->l);
    }
}

/* mul_fft.c:2925-2979 IFFT_radix2_mfa_truncate: inverse of the above, result x 2n
 * for slots 0 .. trunc-1 (true coefficients >= trunc must be zero) */
static void o_ifft_mfa_trunc(octx *c, limb_t **ii, long n, unsigned long w, long n1, long trunc)
{
    long n2 = 2 * n / n1;
    unsigned dr = o_log2(n2), dc = o_log2(n1);
    long tr = trunc / n1;
    for (long s = 0; s < tr; s++) {
        long row = o_revbin(s, dr);
        limb_t **rp = ii + row * n1;
        for (long j = 0; j < n1; j++) {
            long t = o_revbin(j, dc);
            if (j < t) SWAP_PTR(rp[j], rp[t]);
        }
        o_ifft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
    }
    for (long col = 0; col < n1; col++) {
        for (long j = 0; j < n2; j++) {
            long s = o_revbin(j, dr);
            if (j < s) SWAP_PTR(ii[col + j * n1], ii[col + s * n1]);
        }
        o_ifft_trunc_tw(c, ii + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1, tr);
        for (long j = 0; j < tr; j++) o_normmod(ii[col + j * n1], c->l);
    }
}

/* Restatement of MPIR 2.4.0 mpn_mulmod_2expp1 as called at mul_fft.c:3119-3123:
 * r = a b mod 2^N + 1 for normalised a, b; flag bit 0 (1) marks a == 2^N,
 * bit 1 (2) marks b == 2^N.  Writes l limbs and returns the carry limb. */
static limb_t o_mulmod_2expp1(limb_t *r, const limb_t *a, const limb_t *b, int flag,
                              long l, limb_t *tt)
{
    if (flag == 3) {                 /* (-1)(-1) */
        memset(r, 0, (size_t)l * sizeof(limb_t));
        r[0] = 1;
        return 0;
    }
    if (flag) {                      /* 2^N == -1: r = -other */
        const limb_t *o = (flag == 1) ? b : a;
        if (o_is_zero(o, l)) {
            memset(r, 0, (size_t)l * sizeof(limb_t));
            return 0;
        }
        o_neg_n(r, o, l);            /* B^l - o, then + 1 */
        return o_incr(r, l, 1);
    }
    __gmpn_mul_n(tt, a, b, l);       /* lo + hi B^l == lo - hi */
    if (o_sub_n(r, tt, tt + l, l)) return o_incr(r, l, 1);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* L5: new_mpn_mul (mul_fft.c:3190-3265) with the pointwise row fix          */
/* ------------------------------------------------------------------------- */

typedef struct {
    long n, l, sqrt_, j1, j2, trunc, tr;
    unsigned long bits1;
} oparams;

static void o_params(oparams *p, long n1, long n2, unsigned long depth, unsigned long w)
{
    p->n = 1L << depth;
    p->bits1 = ((unsigned long)p->n * w - depth) / 2;
    p->sqrt_ = 1L << (depth / 2);
    p->j1 = (long)((64UL * (unsigned long)n1 - 1) / p->bits1 + 1);
    p->j2 = (long)((64UL * (unsigned long)n2 - 1) / p->bits1 + 1);
    p->trunc = ((p->j1 + p->j2 - 2 + 2 * p->sqrt_) / (2 * p->sqrt_)) * 2 * p->sqrt_;
    p->l = (long)((unsigned long)p->n * w / 64);
    p->tr = p->trunc / p->sqrt_;
}

/* a table of 2n pointers into one block of 2n coefficients (+3 temporaries) */
static limb_t **o_table(long cnt, long l, limb_t **block, octx *c)
{
    limb_t **tab = (limb_t **)malloc((size_t)cnt * sizeof(limb_t *));
    *block = (limb_t *)calloc((size_t)(cnt + 3) * (size_t)(l + 1), sizeof(limb_t));
    for (long i = 0; i < cnt; i++) tab[i] = *block + i * (l + 1);
    if (c) {
        c->l = l;
        c->N = 64UL * (unsigned long)l;
        c->t1 = *block + cnt * (l + 1);
        c->t2 = c->t1 + (l + 1);
        c->t3 = c->t2 + (l + 1);
    }
    return tab;
}

void orc_new_mpn_mul(limb_t *r1, const limb_t *i1, long n1, const limb_t *i2, long n2,
                     unsigned long depth, unsigned long w)
{
    oparams p;
    o_params(&p, n1, n2, depth, w);
    long n = p.n, l = p.l, sq = p.sqrt_;
    octx ca, cb;
    limb_t *ba, *bb;
    limb_t **ii = o_table(2 * n, l, &ba, &ca);
    limb_t **jj = o_table(2 * n, l, &bb, &cb);
    limb_t *tt = (limb_t *)malloc((size_t)(2 * (l + 1)) * sizeof(limb_t));

    long j = o_split_bits(ii, i1, n1, p.bits1, l);
    for (; j < p.trunc; j++) memset(ii[j], 0, (size_t)(l + 1) * sizeof(limb_t));
    o_fft_mfa_trunc(&ca, ii, n, w, sq, p.trunc);

    j = o_split_bits(jj, i2, n2, p.bits1, l);
    for (; j < p.trunc; j++) memset(jj[j], 0, (size_t)(l + 1) * sizeof(limb_t));
    o_fft_mfa_trunc(&cb, jj, n, w, sq, p.trunc);

    /* pointwise over the computed rows; width log2(NR) = depth + 1 - depth/2
     * (the shipped (depth+1)/2 at mul_fft.c:3246 is the SURVEY 0.3 defect) */
    unsigned rw = (unsigned)(depth + 1 - depth / 2);
    for (long s = 0; s < p.tr; s++) {
        long u = o_revbin(s, rw) * sq;
        for (long t = 0; t < sq; t++) {
            long k = u + t;
            int flag = (int)(ii[k][l] + 2 * jj[k][l]);
            ii[k][l] = o_mulmod_2expp1(ii[k], ii[k], jj[k], flag, l, tt);
        }
    }

    o_ifft_mfa_trunc(&ca, ii, n, w, sq, p.trunc);
    for (j = 0; j < p.trunc; j++) {   /* undo the 2n = 2^(depth+1) scaling */
        o_div_2expmod(ii[j], ii[j], l, (unsigned)(depth + 1));
        o_normmod(ii[j], l);
    }
    memset(r1, 0, (size_t)(n1 + n2) * sizeof(limb_t));
    o_combine_bits(r1, ii, p.j1 + p.j2 - 1, p.bits1, l, n1 + n2);

    free(tt);
    free(ii); free(ba);
    free(jj); free(bb);
}

/* ------------------------------------------------------------------------- */
/* L6: the sqrt2 front end new_mpn_mul6 (mul_fft.c:3573-3668)                */
/* ------------------------------------------------------------------------- */

/* r = a * z^i mod p, z the 4n-th root of unity sqrt2^w (z^2 = 2^w), N = n w.
 * i w even: the shift 2^(i w / 2) (FFT_twiddle, mul_fft.c:926, called with (i/2, n, w)
 * for odd w and with (i, 2n, w/2) for even w); i w odd: 2^((i w - 1)/2) sqrt2 with
 * sqrt2 = 2^(3N/4) - 2^(N/4) (FFT_twiddle_sqrt2 :972 / FFT_radix2_butterfly_sqrt2 :591:
 * "multiply by 2^(j + wn/4 + ik), then again by a further 2^(wn/2) and subtract").
 * r must not alias a; t is scratch of l + 1 limbs. */
static void o_mul_root4n(limb_t *r, const limb_t *a, long l, unsigned long i, unsigned long w, limb_t *t)
{
    unsigned long N = 64UL * (unsigned long)l, iw = i * w;
    if ((iw & 1) == 0) {
        o_mul_2exp(r, a, l, iw / 2);
        return;
    }
    unsigned long e = (iw - 1) / 2;
    o_mul_2exp(t, a, l, e + 3 * N / 4);
    o_mul_2exp(r, a, l, e + N / 4);
    o_sub_n(r, t, r, l + 1);
}

/* mul_fft.c:2212-2355 FFT_radix2_mfa_truncate_sqrt2: length-4n truncated transform
 * with root z.  Top level pairs (j, j + 2n) by sum / z^j difference (:2232-2281), then
 * the first half is a full length-2n MFA (:2283-2316) and the second a truncated one
 * over trunc2 = (trunc - 2n)/n1 rows (:2318-2354).  trunc <= 2n (the reference needs
 * trunc > 2n; it indexes ii with trunc2 < 0) leaves the second half unused. */
static void o_fft_mfa_trunc_sqrt2(octx *c, limb_t **ii, long n, unsigned long w, long n1, long trunc)
{
    long l = c->l, n2 = 2 * n / n1;
    long trunc2 = trunc > 2 * n ? (trunc - 2 * n) / n1 : 0;
    unsigned dr = o_log2(n2), dc = o_log2(n1);
    for (long col = 0; col < n1; col++) {
        long j = col;
        for (; j < trunc - 2 * n; j += n1) {          /* (a, b) -> (a + b, z^j (a - b)) */
            o_add_n(c->t1, ii[j], ii[2 * n + j], l + 1);
            o_sub_n(c->t3, ii[j], ii[2 * n + j], l + 1);
            o_mul_root4n(c->t2, c->t3, l, (unsigned long)j, w, ii[2 * n + j]);
            SWAP_PTR(ii[j], c->t1);
            SWAP_PTR(ii[2 * n + j], c->t2);
        }
        if (trunc2)
            for (; j < 2 * n; j += n1)                /* b = 0: z^j a */
                o_mul_root4n(ii[2 * n + j], ii[j], l, (unsigned long)j, w, c->t3);
        o_fft_tw(c, ii + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1);
        for (long r = 0; r < n2; r++) {
            long s = o_revbin(r, dr);
            if (r < s) SWAP_PTR(ii[col + r * n1], ii[col + s * n1]);
        }
    }
    for (long row = 0; row < n2; row++) {
        limb_t **rp = ii + row * n1;
        o_fft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
        for (long k = 0; k < n1; k++) {
            long t = o_revbin(k, dc);
            if (k < t) SWAP_PTR(rp[k], rp[t]);
        }
    }
    ii += 2 * n;
    if (!trunc2) return;
    for (long col = 0; col < n1; col++) {
        o_fft_trunc1_tw(c, ii + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1, trunc2);
        for (long r = 0; r < n2; r++) {
            long s = o_revbin(r, dr);
            if (r < s) SWAP_PTR(ii[col + r * n1], ii[col + s * n1]);
        }
    }
    for (long s = 0; s < trunc2; s++) {
        limb_t **rp = ii + o_revbin(s, dr) * n1;
        o_fft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
        for (long k = 0; k < n1; k++) {
            long t = o_revbin(k, dc);
            if (k < t) SWAP_PTR(rp[k], rp[t]);
        }
    }
}

/* mul_fft.c:2593-2743 IFFT_radix2_mfa_truncate_sqrt2: result x 4n for slots < trunc */
static void o_ifft_mfa_trunc_sqrt2(octx *c, limb_t **ii, long n, unsigned long w, long n1, long trunc)
{
    long l = c->l, n2 = 2 * n / n1;
    long trunc2 = trunc > 2 * n ? (trunc - 2 * n) / n1 : 0;
    unsigned dr = o_log2(n2), dc = o_log2(n1);
    for (long row = 0; row < n2; row++) {             /* first half: full inverse */
        limb_t **rp = ii + row * n1;
        for (long k = 0; k < n1; k++) {
            long t = o_revbin(k, dc);
            if (k < t) SWAP_PTR(rp[k], rp[t]);
        }
        o_ifft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
    }
    for (long col = 0; col < n1; col++) {
        for (long r = 0; r < n2; r++) {
            long s = o_revbin(r, dr);
            if (r < s) SWAP_PTR(ii[col + r * n1], ii[col + s * n1]);
        }
        o_ifft_tw(c, ii + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1);
    }
    limb_t **jj = ii + 2 * n;
    for (long s = 0; s < trunc2; s++) {               /* second half: computed rows */
        limb_t **rp = jj + o_revbin(s, dr) * n1;
        for (long k = 0; k < n1; k++) {
            long t = o_revbin(k, dc);
            if (k < t) SWAP_PTR(rp[k], rp[t]);
        }
        o_ifft(c, rp, 1, n1 / 2, w * (unsigned long)n2);
    }
    for (long col = 0; col < n1; col++) {
        if (trunc2) {
            for (long r = 0; r < trunc2; r++) {
                long s = o_revbin(r, dr);
                if (r < s) SWAP_PTR(jj[col + r * n1], jj[col + s * n1]);
            }
            for (long r = trunc2; r < n2; r++) {      /* x_(u+2n) = 0: z^u (2n x_u) */
                long u = col + r * n1;
                o_mul_root4n(jj[u], ii[u], l, (unsigned long)u, w, c->t3);
            }
            o_ifft_trunc1_tw(c, jj + col, n1, n2 / 2, w * (unsigned long)n1, w, 0, col, 1, trunc2);
        }
        long j = col;
        for (; j < trunc - 2 * n; j += n1) {          /* (a, b) -> a +- z^-j b */
            o_mul_root4n(c->t3, jj[j], l, (unsigned long)(4 * n - j), w, c->t1);
            o_add_n(c->t1, ii[j], c->t3, l + 1);
            o_sub_n(c->t2, ii[j], c->t3, l + 1);
            SWAP_PTR(ii[j], c->t1);
            SWAP_PTR(jj[j], c->t2);
        }
        for (; j < 2 * n; j += n1) o_add_n(ii[j], ii[j], ii[j], l + 1);
    }
}

static void o_params6(oparams *p, long n1, long n2, unsigned long depth, unsigned long w)
{
    o_params(p, n1, n2, depth, w);
    p->bits1 = ((unsigned long)p->n * w - (depth + 1)) / 2;   /* mul_fft.c:3578 */
    p->j1 = (long)((64UL * (unsigned long)n1 - 1) / p->bits1 + 1);
    p->j2 = (long)((64UL * (unsigned long)n2 - 1) / p->bits1 + 1);
    p->trunc = ((p->j1 + p->j2 - 2 + 2 * p->sqrt_) / (2 * p->sqrt_)) * 2 * p->sqrt_;
    p->tr = p->trunc / p->sqrt_;
}

/* mul_fft.c:3573-3668 new_mpn_mul6: length-4n convolution via the sqrt2 transforms,
 * pointwise over the first half and the computed rows of the second (:3621-3648),
 * scaling 2^-(depth+2) (:3654-3658) */
void orc_new_mpn_mul6(limb_t *r1, const limb_t *i1, long n1, const limb_t *i2, long n2,
                      unsigned long depth, unsigned long w)
{
    oparams p;
    o_params6(&p, n1, n2, depth, w);
    long n = p.n, l = p.l, sq = p.sqrt_, n2r = 2 * n / sq;
    octx ca, cb;
    limb_t *ba, *bb;
    limb_t **ii = o_table(4 * n, l, &ba, &ca);
    limb_t **jj = o_table(4 * n, l, &bb, &cb);
    limb_t *tt = (limb_t *)malloc((size_t)(2 * (l + 1)) * sizeof(limb_t));

    o_split_bits(ii, i1, n1, p.bits1, l);              /* the rest of the table is zero (calloc) */
    o_fft_mfa_trunc_sqrt2(&ca, ii, n, w, sq, p.trunc);
    o_split_bits(jj, i2, n2, p.bits1, l);
    o_fft_mfa_trunc_sqrt2(&cb, jj, n, w, sq, p.trunc);

    long trunc2 = p.trunc > 2 * n ? (p.trunc - 2 * n) / sq : 0;
    unsigned rw = o_log2(n2r);
    for (long k = 0; k < 4 * n; k++) {
        if (k >= 2 * n) {
            long s = (k - 2 * n) / sq;                 /* row of the second half */
            if (o_revbin(s, rw) >= trunc2) continue;   /* s = revbin(s'), s' < trunc2 computed */
        }
        o_normmod(ii[k], l);
        o_normmod(jj[k], l);
        int flag = (int)(ii[k][l] + 2 * jj[k][l]);
        ii[k][l] = o_mulmod_2expp1(ii[k], ii[k], jj[k], flag, l, tt);
    }

    o_ifft_mfa_trunc_sqrt2(&ca, ii, n, w, sq, p.trunc);
    for (long j = 0; j < p.trunc; j++) {
        o_div_2expmod(ii[j], ii[j], l, (unsigned)(depth + 2));
        o_normmod(ii[j], l);
    }
    memset(r1, 0, (size_t)(n1 + n2) * sizeof(limb_t));
    o_combine_bits(r1, ii, p.j1 + p.j2 - 1, p.bits1, l, n1 + n2);

    free(tt);
    free(ii); free(ba);
    free(jj); free(bb);
}

void orc_params6(long n1, long n2, unsigned long depth, unsigned long w, long *out)
{
    oparams p;
    o_params6(&p, n1, n2, depth, w);
    out[0] = p.n; out[1] = p.l; out[2] = p.sqrt_; out[3] = p.j1; out[4] = p.j2;
    out[5] = p.trunc; out[6] = (long)p.bits1;
}

/* ------------------------------------------------------------------------- */
/* ctypes-facing wrappers for the tests (flat arrays of (l+1)-limb blocks)   */
/* ------------------------------------------------------------------------- */

void orc_params(long n1, long n2, unsigned long depth, unsigned long w, long *out)
{
    oparams p;
    o_params(&p, n1, n2, depth, w);
    out[0] = p.n; out[1] = p.l; out[2] = p.sqrt_; out[3] = p.j1; out[4] = p.j2;
    out[5] = p.trunc; out[6] = (long)p.bits1;
}

void orc_normmod(limb_t *t, long l) { o_normmod(t, l); }
void orc_mul_2expmod(limb_t *t, const limb_t *a, long l, unsigned d) { o_mul_2expmod(t, a, l, d); }
void orc_div_2expmod(limb_t *t, const limb_t *a, long l, unsigned d) { o_div_2expmod(t, a, l, d); }
void orc_mul_2exp(limb_t *r, const limb_t *a, long l, unsigned long e) { o_mul_2exp(r, a, l, e); }

/* mul_fft.c:303-385 semantics: t = (a + b) B^x, u = (a - b) B^y, 0 <= x, y <= l */
void orc_lshB_sumdiffmod(limb_t *t, limb_t *u, const limb_t *a, const limb_t *b,
                         long l, long x, long y)
{
    limb_t *s = (limb_t *)malloc((size_t)(l + 1) * sizeof(limb_t));
    o_add_n(s, a, b, l + 1);
    o_mul_2exp(t, s, l, 64UL * (unsigned long)x);
    o_sub_n(s, a, b, l + 1);
    o_mul_2exp(u, s, l, 64UL * (unsigned long)y);
    free(s);
}

/* mul_fft.c:394-464 semantics (per its test oracle :3740-3760):
 * t = a / B^x + b / B^y, u = a / B^x - b / B^y, 0 <= x, y < l */
void orc_sumdiff_rshBmod(limb_t *t, limb_t *u, const limb_t *a, const limb_t *b,
                         long l, long x, long y)
{
    unsigned long M = 128UL * (unsigned long)l;
    limb_t *s1 = (limb_t *)malloc((size_t)(2 * (l + 1)) * sizeof(limb_t));
    limb_t *s2 = s1 + (l + 1);
    o_mul_2exp(s1, a, l, (M - 64UL * (unsigned long)x) % M);
    o_mul_2exp(s2, b, l, (M - 64UL * (unsigned long)y) % M);
    o_add_n(t, s1, s2, l + 1);
    o_sub_n(u, s1, s2, l + 1);
    free(s1);
}

limb_t orc_mulmod_2expp1(limb_t *r, const limb_t *a, const limb_t *b, int flag, long l)
{
    limb_t *tt = (limb_t *)malloc((size_t)(2 * l) * sizeof(limb_t));
    limb_t top = o_mulmod_2expp1(r, a, b, flag, l, tt);
    free(tt);
    return top;
}

/* run `kind` on 2n flat coefficients in place:
 *   0 FFT_radix2            (mul_fft.c:786)   length 2n root 2^w
 *   1 IFFT_radix2           (mul_fft.c:1444)
 *   2 truncated FFT, no twiddle (FFT_radix2_truncate_twiddle with c = 0 == FFT_radix2_truncate :1128)
 *   3 truncated IFFT, no twiddle (IFFT_radix2_truncate_twiddle with c = 0 == IFFT_radix2_truncate :1674)
 *   4 FFT_radix2_mfa_truncate  (mul_fft.c:2357) with n1 columns
 *   5 IFFT_radix2_mfa_truncate (mul_fft.c:2925) */
void orc_transform(int kind, limb_t *flat, long n, unsigned long w, long n1, long trunc)
{
    long l = (long)((unsigned long)n * w / 64);
    octx c;
    limb_t *blk;
    limb_t **ii = o_table(2 * n, l, &blk, &c);
    for (long i = 0; i < 2 * n; i++) memcpy(ii[i], flat + i * (l + 1), (size_t)(l + 1) * sizeof(limb_t));
    switch (kind) {
    case 0: o_fft(&c, ii, 1, n, w); break;
    case 1: o_ifft(&c, ii, 1, n, w); break;
    case 2: o_fft_trunc_tw(&c, ii, 1, n, w, 0, 0, 0, 1, trunc); break;
    case 3: o_ifft_trunc_tw(&c, ii, 1, n, w, 0, 0, 0, 1, trunc); break;
    case 4: o_fft_mfa_trunc(&c, ii, n, w, n1, trunc); break;
    case 5: o_ifft_mfa_trunc(&c, ii, n, w, n1, trunc); break;
    }
    for (long i = 0; i < 2 * n; i++) memcpy(flat + i * (l + 1), ii[i], (size_t)(l + 1) * sizeof(limb_t));
    free(ii);
    free(blk);
}

/* split into `count` flat (l+1)-limb blocks (zero beyond the operand) */
long orc_split(limb_t *flat, long count, const limb_t *src, long nlimbs, unsigned long bits, long l)
{
    limb_t **tab = (limb_t **)malloc((size_t)count * sizeof(limb_t *));
    for (long i = 0; i < count; i++) {
        tab[i] = flat + i * (l + 1);
        memset(tab[i], 0, (size_t)(l + 1) * sizeof(limb_t));
    }
    long len = (long)((64UL * (unsigned long)nlimbs - 1) / bits + 1);
    if (len > count) len = count;
    for (long j = 0; j < len; j++) {
        unsigned long start = (unsigned long)j * bits, total = 64UL * (unsigned long)nlimbs;
        unsigned long cnt = (start + bits <= total) ? bits : total - start;
        o_extract_bits(tab[j], src, nlimbs, start, cnt);
    }
    free(tab);
    return len;
}

void orc_combine(limb_t *res, const limb_t *flat, long len, unsigned long bits, long l, long total)
{
    limb_t **tab = (limb_t **)malloc((size_t)len * sizeof(limb_t *));
    for (long i = 0; i < len; i++) tab[i] = (limb_t *)(flat + i * (l + 1));
    memset(res, 0, (size_t)total * sizeof(limb_t));
    o_combine_bits(res, tab, len, bits, l, total);
    free(tab);
}

/* GMP mpn_mul, the reference's integration-test oracle (mul_fft.c:5542) */
void orc_gmp_mul(limb_t *r, const limb_t *a, long na, const limb_t *b, long nb)
{
    if (na >= nb) __gmpn_mul(r, a, na, b, nb);
    else __gmpn_mul(r, b, nb, a, na);
}

/* splitmix64-seeded xoshiro256** (BASELINE.md "Synthetic inputs") */
static uint64_t o_rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

void orc_fill_random(limb_t *buf, long cnt, uint64_t seed)
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
        buf[i] = o_rotl(s[1] * 5, 7) * 9;
        uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t;
        s[3] = o_rotl(s[3], 45);
    }
}
