// bpass.hip -- instantiations of the big-coefficient LDS-resident passes (bkernels.hpp),
// limb-aligned rotations only (GEN = false); bpass_gen.hip holds the general ones.
#include "bkernels.hpp"
#include "bdispatch.hpp"

static bp_fn bp_table[2][BP_MAXLOGG + 1] = {
    {nullptr, k_bpass<1, 0, false>, k_bpass<2, 0, false>, k_bpass<3, 0, false>, k_bpass<4, 0, false>},
    {nullptr, k_bpass<1, 1, false>, k_bpass<2, 1, false>, k_bpass<3, 1, false>, k_bpass<4, 1, false>},
};

bp_fn bp_get(int logg, int dir)
{
    if (logg < 1 || logg > BP_MAXLOGG || dir < 0 || dir > 1) return nullptr;
    return bp_table[dir][logg];
}
