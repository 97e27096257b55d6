// pdispatch.hpp -- host-side view of the nested negacyclic pointwise kernel (pkernels.hpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

typedef void (*pw_fn)(uint64_t *, uint64_t *, int *, const uint64_t *, const uint64_t *, const int *, int,
                      uint64_t *, uint64_t *, int *, unsigned long long *);

// k_pwss<M, lk, fuse> (M = inner coefficient limbs, 2^lk pieces; fuse 1: the row DIF's last
// level fused into the load, product to the C arrays), nullptr if not built
pw_fn pw_get(int M, int lk, int fuse = 0);
size_t pw_lds(int M, int K, int l);
// k_pw2<M, lk, fuse>: the same with two threads per piece (p2kernels.hpp; 2^(lk+1) threads)
pw_fn pw2_get(int M, int lk, int fuse = 0);
size_t pw2_lds(int M, int K, int l);

// Inner ring for a product mod 2^(64 l) + 1 cut into K = 2^lk pieces: the smallest M
// (limbs) with 64 M >= 2 (64 l / K) + lk + 2 and 64 M a multiple of K (theta = 2^(64 M / K)).
inline int pw_inner_limbs(long l, int lk)
{
    const long K = 1L << lk, B = 64 * l / K;
    const long need = 2 * B + lk + 2;
    const long step = K / 64 > 1 ? K / 64 : 1;   // M multiple of K / 64
    long M = (need + 63) / 64;
    M = (M + step - 1) / step * step;
    return (int)M;
}
