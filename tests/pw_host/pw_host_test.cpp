// Host-side unit test of the nested-pointwise arithmetic (mpir-fft_amd/csrc/pkernels.hpp):
// pw_combine (rotated add in R' = Z/(2^N'+1)), pw_mulmod (inner product) and pw_canon,
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
    constexpr int K = 4;
    mpz_t p, a, b, want, got, e2; mpz_inits(p, a, b, want, got, e2, NULL);
    mpz_set_ui(p, 1); mpz_mul_2exp(p, p, 64 * M); mpz_add_ui(p, p, 1);
    int bad = 0;
    for (int it = 0; it < 20000; ++it) {
        u64 L[M], X[M * K]; int T = (int)(rng() % 401) - 200, Tq = (int)(rng() % 401) - 200;
        for (int j = 0; j < M; ++j) L[j] = rng();
        int TT[K];
        for (int j = 0; j < M * K; ++j) X[j] = rng();
        for (int j = 0; j < K; ++j) TT[j] = Tq;
        int q = rng() % K; unsigned E = rng() % (128 * M); int alpha = (int)(rng() % 3) - 1;
        u64 Xq[M]; for (int j = 0; j < M; ++j) Xq[j] = X[j * K + q];
        tovals<M>(a, L, T); tovals<M>(b, Xq, Tq);
        mpz_ui_pow_ui(e2, 2, E); mpz_mul(want, b, e2); mpz_mul_si(a, a, alpha); mpz_add(want, want, a); mpz_mod(want, want, p);
        pw_combine<M>(L, T, alpha, X, TT, K, q, E);
        tovals<M>(got, L, T); mpz_mod(got, got, p);
        if (mpz_cmp(got, want)) { if (bad++ < 5) printf("combine mismatch it=%d E=%u alpha=%d\n", it, E, alpha); }
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
    return bad + bad0;
}

int main()
{
    int bad = run<12>() + run<20>() + run<24>();
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
