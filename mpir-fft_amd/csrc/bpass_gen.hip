// bpass_gen.hip -- k_bpass instantiations for passes with sub-limb rotations (GEN = true)
#include "bkernels.hpp"
#include "bdispatch.hpp"

static bp_fn bp_table_gen[2][BP_MAXLOGG + 1] = {
    {nullptr, k_bpass<1, 0, true>, k_bpass<2, 0, true>, k_bpass<3, 0, true>, k_bpass<4, 0, true>},
    {nullptr, k_bpass<1, 1, true>, k_bpass<2, 1, true>, k_bpass<3, 1, true>, k_bpass<4, 1, true>},
};

bp_fn bp_get_gen(int logg, int dir)
{
    if (logg < 1 || logg > BP_MAXLOGG || dir < 0 || dir > 1) return nullptr;
    return bp_table_gen[dir][logg];
}
