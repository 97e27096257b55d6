// wave kernels, 64 < l <= 128 limbs
#define WU 2
#define WFN 0
#define WF false
#define WMAXLOGG 3
#include "wpass_impl.hpp"
