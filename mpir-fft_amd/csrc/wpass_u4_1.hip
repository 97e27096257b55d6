// wave kernels, 192 < l <= 256 limbs (l == 256)
#define WU 4
#define WFN 1
#define WF true
#define WMAXLOGG 3
#include "wpass_impl.hpp"
