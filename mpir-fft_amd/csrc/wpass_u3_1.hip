// wave kernels, 128 < l <= 192 limbs (l == 192)
#define WU 3
#define WFN 1
#define WF true
#define WMAXLOGG 3
#include "wpass_impl.hpp"
