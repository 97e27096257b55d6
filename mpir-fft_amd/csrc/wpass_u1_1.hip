// wave kernels, 0 < l <= 64 limbs (l == 64)
#define WU 1
#define WFN 1
#define WF true
#define WMAXLOGG 4
#include "wpass_impl.hpp"
