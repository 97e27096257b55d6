/*
 * time_mul.c -- the reference's own driver shape for new_mpn_mul, linked against
 * libmpfft.so instead of mul_fft.c: a C caller that includes include/mpfft.h and
 * calls the exported new_mpn_mul symbol directly (the drop-in boundary).
 *
 * Mirrors time_mul (/root/reference/mul_fft.c:5288-5324): random operands from
 * GMP's default generator (mpz_urandomb, as mpn_urandomb there), `iters` calls of
 * new_mpn_mul(r1, i1, n, i2, n, depth, w).  Unlike the reference (which times
 * externally and checks nothing -- and whose hard-coded 8364032-bit size does not
 * fit depth 10, w 3: j1 + j2 - 1 = 10925 > 2^11), every product is checked
 * against GMP mpn_mul, the reference's integration-test oracle (mul_fft.c:5542).
 *
 * usage: time_mul [depth w limbs iters]     -> prints "ok <ms per call>" or "MISMATCH"
 *        time_mul --mul6 depth w limbs iters -> the same through new_mpn_mul6 (the sqrt2
 *                                              front end, mul_fft.c:3573; test_mul4 :5559)
 *        time_mul --devices 0,1,2,3 depth w limbs iters
 *                                           -> mpfft_mul_multi: the product column-sharded over
 *                                              those HIP devices from this one process
 *        time_mul --bad                     -> invalid parameters: new_mpn_mul must abort
 * With MPFFT_DEVICES=0,1,...,7 in the environment the plain new_mpn_mul calls shard too (the
 * library's device policy) -- the caller stays unmodified.
 * Built by __graft_entry__.build() (gcc, -lmpfft -lgmp); run by tests/test_c_abi.py.
 */
#include <gmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpfft.h"

static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static int ndevs;
static int devs[64];

/* new_mpn_mul's signature over mpfft_mul_multi with the --devices list */
static void mul_multi(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1, mp_limb_t *i2, mp_size_t n2, mp_bitcnt_t depth,
                      mp_bitcnt_t w)
{
    int rc = mpfft_mul_multi(r1, i1, n1, i2, n2, depth, w, ndevs, devs);
    if (rc) {
        fprintf(stderr, "mpfft_mul_multi: %s\n", mpfft_strerror(rc));
        exit(2);
    }
}

static void random_limbs(mp_limb_t *dst, mp_size_t n, gmp_randstate_t st)
{
    mpz_t z;
    mpz_init(z);
    mpz_urandomb(z, st, (mp_bitcnt_t)n * GMP_LIMB_BITS);
    size_t cnt = 0;
    memset(dst, 0, n * sizeof(mp_limb_t));
    mpz_export(dst, &cnt, -1, sizeof(mp_limb_t), 0, 0, z);
    mpz_clear(z);
}

int main(int argc, char **argv)
{
    if (argc > 1 && !strcmp(argv[1], "--bad")) {
        mp_limb_t a[4] = {1, 2, 3, 4}, r[8];
        new_mpn_mul(r, a, 4, a, 4, 5, 3);   /* n*w = 96 is not a whole number of limbs */
        printf("returned\n");               /* unreachable: new_mpn_mul aborts */
        return 0;
    }
    int six = argc > 1 && !strcmp(argv[1], "--mul6");
    if (six) {
        argv++;
        argc--;
    }
    if (argc > 2 && !strcmp(argv[1], "--devices")) {
        for (char *q = argv[2]; *q && ndevs < 64;) {
            devs[ndevs++] = (int)strtol(q, &q, 10);
            if (*q == ',') q++;
        }
        argv += 2;
        argc -= 2;
    }
    void (*mul)(mp_limb_t *, mp_limb_t *, mp_size_t, mp_limb_t *, mp_size_t, mp_bitcnt_t, mp_bitcnt_t) =
        six ? new_mpn_mul6 : ndevs ? mul_multi : new_mpn_mul;
    mp_bitcnt_t depth = argc > 4 ? strtoul(argv[1], 0, 0) : 10;
    mp_bitcnt_t w = argc > 4 ? strtoul(argv[2], 0, 0) : 3;
    mp_size_t n = argc > 4 ? strtol(argv[3], 0, 0) : 24000;
    long iters = argc > 4 ? strtol(argv[4], 0, 0) : 10;

    gmp_randstate_t state;
    gmp_randinit_default(state);
    mp_limb_t *i1 = malloc(6 * n * sizeof(mp_limb_t));
    mp_limb_t *i2 = i1 + n, *r1 = i2 + n, *r2 = r1 + 2 * n;
    random_limbs(i1, n, state);
    random_limbs(i2, n, state);

    mul(r1, i1, n, i2, n, depth, w);   /* warm-up: device context + workspace */
    double t0 = now_ms();
    for (long i = 0; i < iters; i++) mul(r1, i1, n, i2, n, depth, w);
    double per = (now_ms() - t0) / (iters > 0 ? iters : 1);

    mpn_mul(r2, i1, n, i2, n);
    if (memcmp(r1, r2, 2 * n * sizeof(mp_limb_t))) {
        printf("MISMATCH depth=%lu w=%lu n=%ld\n", (unsigned long)depth, (unsigned long)w, (long)n);
        return 1;
    }
    printf("ok %.3f ms per %s (depth=%lu w=%lu n1=n2=%ld, host pointers, H2D+D2H included; devices=%d)\n", per,
           six ? "new_mpn_mul6" : ndevs ? "mpfft_mul_multi" : "new_mpn_mul", (unsigned long)depth, (unsigned long)w,
           (long)n, ndevs ? ndevs : six ? 1 : mpfft_last_ngpus());
    free(i1);
    gmp_randclear(state);
    return 0;
}
