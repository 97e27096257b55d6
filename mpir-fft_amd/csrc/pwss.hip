// pwss.hip -- instantiations of the nested negacyclic pointwise kernel (pkernels.hpp)
#include "pkernels.hpp"
#include "pdispatch.hpp"

pw_fn pw_get(int M, int lk, int fuse)
{
    if (M == 10 && lk == 8) return fuse == 2 ? nullptr : fuse ? k_pwss<10, 8, 1> : k_pwss<10, 8, 0>;   // l = 1024
    if (M == 18 && lk == 8) return fuse == 2 ? k_pwss<18, 8, 2> : fuse ? k_pwss<18, 8, 1> : k_pwss<18, 8, 0>;   // l = 2048
    if (M == 20 && lk == 9) return fuse == 2 ? k_pwss<20, 9, 2> : fuse ? k_pwss<20, 9, 1> : k_pwss<20, 9, 0>;   // l = 4096
    return nullptr;
}

size_t pw_lds(int M, int K, int l) { return pw_lds_bytes(M, K, l); }
