// pwss.hip -- instantiations of the nested negacyclic pointwise kernel (pkernels.hpp)
#include "pkernels.hpp"
#include "pdispatch.hpp"

pw_fn pw_get(int M, int lk, int fuse)
{
    if (M == 12 && lk == 8) return fuse ? k_pwss<12, 8, 1> : k_pwss<12, 8, 0>;
    if (M == 20 && lk == 8) return fuse ? k_pwss<20, 8, 1> : k_pwss<20, 8, 0>;
    if (M == 24 && lk == 9) return fuse ? k_pwss<24, 9, 1> : k_pwss<24, 9, 0>;
    return nullptr;
}

size_t pw_lds(int M, int K, int l) { return pw_lds_bytes(M, K, l); }
