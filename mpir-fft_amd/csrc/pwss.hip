// pwss.hip -- instantiations of the nested negacyclic pointwise kernel (pkernels.hpp)
#include "pkernels.hpp"
#include "pdispatch.hpp"

pw_fn pw_get(int M)
{
    switch (M) {
    case 12: return k_pwss<12>;
    case 20: return k_pwss<20>;
    case 24: return k_pwss<24>;
    }
    return nullptr;
}

size_t pw_lds(int M, int K, int l) { return pw_lds_bytes(M, K, l); }
