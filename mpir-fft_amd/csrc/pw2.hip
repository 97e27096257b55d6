// pw2.hip -- instantiations of the two-threads-per-piece nested negacyclic pointwise (p2kernels.hpp)
#include "p2kernels.hpp"
#include "pdispatch.hpp"

pw_fn pw2_get(int M, int lk, int fuse)
{
    if (M == 12 && lk == 8) return fuse ? k_pw2<12, 8, 1> : k_pw2<12, 8, 0>;
    if (M == 20 && lk == 8) return fuse ? k_pw2<20, 8, 1> : k_pw2<20, 8, 0>;
    if (M == 24 && lk == 9) return fuse ? k_pw2<24, 9, 1> : k_pw2<24, 9, 0>;
    return nullptr;
}

size_t pw2_lds(int M, int K, int l) { return pw2_lds_bytes(M, K, l); }
