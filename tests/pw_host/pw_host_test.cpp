// Host-side unit test of the nested-pointwise arithmetic (mpir-fft_amd/csrc/pkernels.hpp):
// pw_norm + pw_combine (rotated add in R' = Z/(2^N'+1)), pw_mulmod (inner product) and pw_canon,
// each against GMP mpz on random operands.  The same source runs on the GPU inside
// k_pwss; these functions are __host__ __device__ so the CPU suite can pin them.
// Built by __graft_entry__.build() (tests/pw_host/Makefile), run by tests/test_pw_host.py.
#include "pkernels.hpp"
#include <gmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <random>
static std::mt19937_64 rng(7);
template <int M> void tovals(mpz_t z, const u64 *L, int T) {
    mpz_import(z, M, -1, 8, 0, 0, L);
    mpz_t t; mpz_init_set_si(t, T); mpz_mul_2exp(t, t, 64 * M); mpz_add(z, z, t); mpz_clear(t);
}
template <int M> int run() {
    constexpr int LK = 2, K = 1 << LK;
    mpz_t p, a, b, want, got, e2; mpz_inits(p, a, b, want, got, e2, NULL);
    mpz_set_ui(p, 1); mpz_mul_2exp(p, p, 64 * M); mpz_add_ui(p, p, 1);
    int bad = 0;
    for (int it = 0; it < 20000; ++it) {
        // own value (L, T); partner q published as words (pw_publish's layout, 2M + 2 rows)
        u64 L[M], Lq[M]; int T = (int)(rng() % 401) - 200, Tq = (int)(rng() % 401) - 200;
        for (int j = 0; j < M; ++j) { L[j] = rng(); Lq[j] = rng(); }
        if (it % 7 == 3) for (int j = 0; j < M; ++j) Lq[j] = it % 2 ? 0 : ~0ull;   // pw_norm wraps
        int q = rng() % K; unsigned E = it % 13 == 0 ? (unsigned)(rng() % 4) * 64 * M / 2 : rng() % (128 * M);
        int alpha = (int)(rng() % 3) - 1, S = (int)(rng() & 1), Sq = (int)(rng() & 1);
        tovals<M>(b, Lq, Tq);
        if (it % 3) Tq = pw_norm<M>(Lq, Tq);   // the published form (top almost always -1)
        u64 chk; { mpz_t c2; mpz_init(c2); tovals<M>(c2, Lq, Tq); mpz_sub(c2, c2, b); mpz_mod(c2, c2, p);
                   chk = mpz_sgn(c2); mpz_clear(c2); }
        if (chk) { if (bad++ < 5) printf("norm mismatch it=%d\n", it); }
        u32 Xw[(2 * M + 2) * K]; int TT[K];
        for (int j = 0; j < (2 * M + 2) * K; ++j) Xw[j] = (u32)rng();
        for (int j = 0; j < M; ++j) { Xw[2 * j * K + q] = (u32)Lq[j]; Xw[(2 * j + 1) * K + q] = (u32)(Lq[j] >> 32); }
        TT[q] = 2 * Tq + Sq;
        // represented values carry a sign flag: (-1)^S (L + T 2^N')
        tovals<M>(a, L, T); if (S) mpz_neg(a, a); if (Sq) mpz_neg(b, b);
        mpz_ui_pow_ui(e2, 2, E); mpz_mul(want, b, e2); mpz_mul_si(a, a, alpha); mpz_add(want, want, a); mpz_mod(want, want, p);
        pw_combine<M, LK>(L, T, S, alpha, Xw, TT[q], q, E);
        tovals<M>(got, L, T); if (S) mpz_neg(got, got); mpz_mod(got, got, p);
        if (mpz_cmp(got, want)) { if (bad++ < 5) printf("combine mismatch it=%d E=%u alpha=%d Tq=%d\n", it, E, alpha, Tq); }
    }
    printf("M=%d combine bad=%d\n", M, bad);
    int bad0 = bad;
    bad = 0;
    for (int it = 0; it < 2000; ++it) {
        u64 La[M], Lb[M], Z[M]; int T;
        for (int j = 0; j < M; ++j) { La[j] = rng(); Lb[j] = rng(); }
        if (it % 5 == 1) for (int j = 0; j < M; ++j) La[j] = Lb[j] = ~0ull;   // 2^N' - 1: every column at its maximum
        if (it % 5 == 2) for (int j = 0; j < M; ++j) La[j] = ~0ull;
        int ta = it % 7 == 0, tb = it % 11 == 0;
        if (ta) for (int j = 0; j < M; ++j) La[j] = 0;
        if (tb) for (int j = 0; j < M; ++j) Lb[j] = 0;
        tovals<M>(a, La, ta); tovals<M>(b, Lb, tb); mpz_mul(want, a, b); mpz_mod(want, want, p);
        pw_mulmod<M>(Z, T, La, ta, Lb, tb);
        tovals<M>(got, Z, T); mpz_mod(got, got, p);
        if (mpz_cmp(got, want)) { if (bad++ < 5) printf("mulmod mismatch it=%d\n", it); }
        int Tc = (int)(rng() % 2000001) - 1000000;
        u64 Lc[M]; for (int j = 0; j < M; ++j) Lc[j] = rng();
        tovals<M>(a, Lc, Tc); mpz_mod(want, a, p);
        int c = pw_canon<M>(Lc, Tc);
        tovals<M>(got, Lc, c);
        if (mpz_cmp(got, want)) { if (bad++ < 5) printf("canon mismatch it=%d\n", it); }
    }
    printf("M=%d mulmod/canon bad=%d\n", M, bad);
    int bad1 = bad;
    bad = 0;
    // pw_sqrt2: (2^(N'/2) - 1) x, and its square 2^(N'/2) (2^(N'/2) - 1)^2 == 2 (the sqrt 2
    // identity the odd negacyclic weights rely on, mul_fft.c:579-640)
    mpz_t h; mpz_init(h);
    for (int it = 0; it < 20000; ++it) {
        u64 L[M]; int T = (int)(rng() % 9) - 4;
        for (int j = 0; j < M; ++j) L[j] = it % 9 == 4 ? (it % 2 ? ~0ull : 0ull) : rng();
        tovals<M>(a, L, T);
        mpz_set_ui(h, 1); mpz_mul_2exp(h, h, 32 * M); mpz_sub_ui(h, h, 1);
        mpz_mul(want, a, h); mpz_mod(want, want, p);
        pw_sqrt2<M>(L, T);
        tovals<M>(got, L, T); mpz_mod(got, got, p);
        if (mpz_cmp(got, want)) { if (bad++ < 5) printf("sqrt2 mismatch it=%d\n", it); }
        if (T < -8 || T > 8) { if (bad++ < 5) printf("sqrt2 top out of range T=%d\n", T); }
        if (it == 0) {   // 2^(N'/4) (2^(N'/2) - 1) squared is 2
            mpz_set_ui(a, 1); mpz_mul_2exp(a, a, 16 * M); mpz_mul(a, a, h); mpz_mul(a, a, a); mpz_mod(a, a, p);
            if (mpz_cmp_ui(a, 2)) { ++bad; printf("sqrt2 identity fails\n"); }
        }
    }
    mpz_clear(h);
    printf("M=%d sqrt2 bad=%d\n", M, bad);
    return bad + bad0 + bad1;
}

int main()
{
    int bad = run<10>() + run<18>() + run<20>();
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
