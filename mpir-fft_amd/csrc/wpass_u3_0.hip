// wave kernels, 128 < l <= 192 limbs
#define WU 3
#define WFN 0
#define WF false
#define WMAXLOGG 3
#include "wpass_impl.hpp"
