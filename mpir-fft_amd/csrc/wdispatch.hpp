// wdispatch.hpp -- host-side view of the wave-owned kernels (wkernels.hpp), which are
// instantiated per limbs-per-lane U in their own translation units (wpass_u*.hip) so
// the library builds in parallel.
#pragma once
#include <stdint.h>

struct PassArgs;
struct PairArgs;

#define WPB 4   // waves per workgroup (independent waves sharing a launch)

// LDS staging slots per wave: about 8 KiB of 2l-digit buffers (l <= 64 U), at most G/2
#define LP_MAXLOGG 5   // k_lpass: 2^LOGG / 2 waves <= 16

__host__ __device__ constexpr int wv_stage_slots(int G, int U)
{
    return (G > 1 ? G / 2 : 1) < (8 / U > 1 ? 8 / U : 1) ? (G > 1 ? G / 2 : 1) : (8 / U > 1 ? 8 / U : 1);
}

typedef void (*wv_pass_fn)(PassArgs);
typedef void (*wv_pair_fn)(PairArgs);
typedef void (*wv_scale_fn)(uint64_t *, uint64_t *, int *, int, uint64_t, uint64_t, long);

struct WvFns {
    wv_pass_fn (*pass)(int logg, int dir);   // nullptr when logg > maxlogg
    wv_pair_fn pair;
    wv_scale_fn scale;
    int maxlogg;                              // largest radix-2^logg pass without register spills
    wv_pass_fn (*lpass)(int logg, int dir);   // LDS-resident passes (lkernels.hpp), logg <= 5
};

WvFns wv_fns_u1_0();
WvFns wv_fns_u1_1();
WvFns wv_fns_u2_0();
WvFns wv_fns_u2_1();
WvFns wv_fns_u3_0();
WvFns wv_fns_u3_1();
WvFns wv_fns_u4_0();
WvFns wv_fns_u4_1();
