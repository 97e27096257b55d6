// wave kernels, 0 < l <= 64 limbs
#define WU 1
#define WFN 0
#define WF false
#define WMAXLOGG 4
#include "wpass_impl.hpp"
