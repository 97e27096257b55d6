// rpass_p4.hip -- k_rpass instantiations for l = 4096 limbs (rkernels.hpp)
#include "rkernels.hpp"

rp_fn rp_get_p4(int logg, int dir, int mode)
{
    static const rp_fn tab[2][16][4] = {
        {
            {nullptr, k_rpass<1, 4, 0, 0>, k_rpass<2, 4, 0, 0>, k_rpass<3, 4, 0, 0>},
            {nullptr, k_rpass<1, 4, 0, 1>, k_rpass<2, 4, 0, 1>, k_rpass<3, 4, 0, 1>},
            {nullptr, k_rpass<1, 4, 0, 2>, k_rpass<2, 4, 0, 2>, k_rpass<3, 4, 0, 2>},
            {nullptr, k_rpass<1, 4, 0, 3>, k_rpass<2, 4, 0, 3>, k_rpass<3, 4, 0, 3>},
            {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {},
        },
        {
            {nullptr, k_rpass<1, 4, 1, 0>, k_rpass<2, 4, 1, 0>, k_rpass<3, 4, 1, 0>},
            {nullptr, k_rpass<1, 4, 1, 1>, k_rpass<2, 4, 1, 1>, k_rpass<3, 4, 1, 1>},
            {nullptr, k_rpass<1, 4, 1, 2>, k_rpass<2, 4, 1, 2>, k_rpass<3, 4, 1, 2>},
            {nullptr, k_rpass<1, 4, 1, 3>, k_rpass<2, 4, 1, 3>, k_rpass<3, 4, 1, 3>},
            {nullptr, k_rpass<1, 4, 1, 4>, k_rpass<2, 4, 1, 4>, k_rpass<3, 4, 1, 4>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 4, 1, 6>, k_rpass<2, 4, 1, 6>, k_rpass<3, 4, 1, 6>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 4, 1, 10>, k_rpass<2, 4, 1, 10>, k_rpass<3, 4, 1, 10>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 4, 1, 14>, k_rpass<2, 4, 1, 14>, k_rpass<3, 4, 1, 14>},
            {nullptr, nullptr, nullptr, nullptr},
        },
    };
    if (logg < 1 || logg > 3 || dir < 0 || dir > 1 || mode < 0 || mode > 15) return nullptr;
    return tab[dir][mode][logg];
}

rp_pair_fn rp_chain_get_p4(int nb)
{
    static const rp_pair_fn tab[4] = {nullptr, k_rchain<4, 1>, k_rchain<4, 2>, k_rchain<4, 3>};
    return nb >= 1 && nb <= 3 ? tab[nb] : nullptr;
}

rp_pair_fn rp_pair_get_p4(int op)
{
    static const rp_pair_fn tab[6] = {k_rpair<4, OP_DOUBLE>, k_rpair<4, OP_HALFADD>, k_rpair<4, OP_FILL>,
                                      k_rpair<4, OP_FIX>, k_rpair<4, OP_TWOXMY>, k_rpair<4, OP_IBFLY>};
    return op >= 0 && op < 6 ? tab[op] : nullptr;
}

void (*rp_scale_get_p4(int nt))(u64 *, u64 *, int *, u32, u32, u32, u32, u32)
{
    return nt == 256 ? k_rscale<4, 256> : k_rscale<4>;
}
