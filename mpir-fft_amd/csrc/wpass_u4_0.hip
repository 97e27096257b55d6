// wave kernels, 192 < l <= 256 limbs
#define WU 4
#define WFN 0
#define WF false
#define WMAXLOGG 3
#include "wpass_impl.hpp"
