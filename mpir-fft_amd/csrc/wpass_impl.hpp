// wpass_impl.hpp -- instantiates the wave kernels for one (U, F) (define WU, WF, WMAXLOGG first)
#include "lkernels.hpp"

#define WV_NAME2(u, f) wv_fns_u##u##_##f
#define WV_NAME(u, f) WV_NAME2(u, f)

static wv_pass_fn wv_get_pass(int logg, int dir)
{
    if (dir == 0) {
        switch (logg) {
        case 1: return k_wpass<WU, WF, 1, 0>;
        case 2: return k_wpass<WU, WF, 2, 0>;
        case 3: return k_wpass<WU, WF, 3, 0>;
#if WMAXLOGG >= 4
        case 4: return k_wpass<WU, WF, 4, 0>;
#endif
        }
    } else {
        switch (logg) {
        case 1: return k_wpass<WU, WF, 1, 1>;
        case 2: return k_wpass<WU, WF, 2, 1>;
        case 3: return k_wpass<WU, WF, 3, 1>;
#if WMAXLOGG >= 4
        case 4: return k_wpass<WU, WF, 4, 1>;
#endif
        }
    }
    return nullptr;
}

static wv_pass_fn lp_get_pass(int logg, int dir)
{
    if (dir == 0) {
        switch (logg) {
        case 1: return k_lpass<WU, WF, 1, 0>;
        case 2: return k_lpass<WU, WF, 2, 0>;
        case 3: return k_lpass<WU, WF, 3, 0>;
        case 4: return k_lpass<WU, WF, 4, 0>;
        case 5: return k_lpass<WU, WF, 5, 0>;
        }
    } else {
        switch (logg) {
        case 1: return k_lpass<WU, WF, 1, 1>;
        case 2: return k_lpass<WU, WF, 2, 1>;
        case 3: return k_lpass<WU, WF, 3, 1>;
        case 4: return k_lpass<WU, WF, 4, 1>;
        case 5: return k_lpass<WU, WF, 5, 1>;
        }
    }
    return nullptr;
}

WvFns WV_NAME(WU, WFN)()
{
    WvFns f;
    f.pass = wv_get_pass;
    f.pair = k_wpair<WU, WF>;
    f.scale = k_wscale<WU, WF>;
    f.maxlogg = WMAXLOGG;
    f.lpass = lp_get_pass;
    return f;
}
