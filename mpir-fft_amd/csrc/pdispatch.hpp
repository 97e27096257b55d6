// pdispatch.hpp -- host-side view of the nested negacyclic pointwise kernel (pkernels.hpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

typedef void (*pw_fn)(uint64_t *, uint64_t *, int *, const uint64_t *, const uint64_t *, const int *, int,
                      uint64_t *, uint64_t *, int *, unsigned long long *);

// k_pwss<M, lk, fuse> (M = inner coefficient limbs, 2^lk pieces; fuse 1: the row DIF's last
// level fused into the load, product to the C arrays; fuse 2: the last two levels, slot quads
// -- their pieces are 4x the inputs', so the plan checks 64 M >= 2 B + lk + 6), nullptr if
// not built
pw_fn pw_get(int M, int lk, int fuse = 0);
size_t pw_lds(int M, int K, int l);

// Inner ring for a product mod 2^(64 l) + 1 cut into K = 2^lk pieces: the smallest even M
// (limbs) with 64 M >= 2 (64 l / K) + lk + 4: the pair-fused inputs (pieces of x0 +- x1) are
// below 2^(B+1) (1 + 2^-64) in magnitude, so |c_t| < K 2^(2B+2) (1 + 2^-62) < 2^(N'-1)
// and 2 (64 M) a multiple of K (omega = 2^(128 M / K); theta may need sqrt 2: pw_sqrt2).
inline int pw_inner_limbs(long l, int lk)
{
    const long K = 1L << lk, B = 64 * l / K;
    const long need = 2 * B + lk + 4;
    long step = K / 128 > 2 ? K / 128 : 2;   // M even, 128 M multiple of K
    long M = (need + 63) / 64;
    M = (M + step - 1) / step * step;
    return (int)M;
}
