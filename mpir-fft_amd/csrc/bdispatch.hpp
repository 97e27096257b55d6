// bdispatch.hpp -- host-side view of the big-coefficient passes (bkernels.hpp, bpass.hip)
#pragma once
#include <stddef.h>

struct PassArgs;
typedef void (*bp_fn)(PassArgs);

#define BP_MAXLOGG 4          // G <= 16 coefficients per workgroup
#define BP_WAVES 16           // at most (G l <= 16384 limbs)
#define BP_RMAX 8             // rows of 64 limbs per wave per level: a wave owns 8 rows of one pair
#define BP_SB 4               // rows per wave in flight in the store phase
#define BP_LB 8               // 16-byte loads in flight per thread in the load phase
#define BP_LDS_MAX (160 * 1024)

bp_fn bp_get(int logg, int dir);       // k_bpass<logg, dir, false>: every rotation limb-aligned
bp_fn bp_get_gen(int logg, int dir);   // k_bpass<logg, dir, true>: general rotations

// waves of a k_bpass workgroup: (G/2 pairs) x (l/64 rows) / BP_RMAX rows per wave
inline int bp_waves(int l, int logg) { return (1 << (logg - 1)) * (l / 64) / BP_RMAX; }

// LDS of a k_bpass group of G coefficients of l limbs: G slots of 9 l bytes + carry limbs
inline size_t bp_lds_need(int l, int G) { return (size_t)G * (((size_t)l * 9 + 15) / 16 * 16) + 16 * (size_t)G; }
