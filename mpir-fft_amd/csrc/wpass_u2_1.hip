// wave kernels, 64 < l <= 128 limbs (l == 128)
#define WU 2
#define WFN 1
#define WF true
#define WMAXLOGG 3
#include "wpass_impl.hpp"
