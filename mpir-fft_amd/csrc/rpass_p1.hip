// rpass_p1.hip -- k_rpass instantiations for l = 1024 limbs (rkernels.hpp)
#include "rkernels.hpp"

rp_fn rp_get_p1(int logg, int dir, int mode)
{
    static const rp_fn tab[2][16][4] = {
        {
            {nullptr, k_rpass<1, 1, 0, 0>, k_rpass<2, 1, 0, 0>, k_rpass<3, 1, 0, 0>},
            {nullptr, k_rpass<1, 1, 0, 1>, k_rpass<2, 1, 0, 1>, k_rpass<3, 1, 0, 1>},
            {nullptr, k_rpass<1, 1, 0, 2>, k_rpass<2, 1, 0, 2>, k_rpass<3, 1, 0, 2>},
            {nullptr, k_rpass<1, 1, 0, 3>, k_rpass<2, 1, 0, 3>, k_rpass<3, 1, 0, 3>},
            {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {}, {},
        },
        {
            {nullptr, k_rpass<1, 1, 1, 0>, k_rpass<2, 1, 1, 0>, k_rpass<3, 1, 1, 0>},
            {nullptr, k_rpass<1, 1, 1, 1>, k_rpass<2, 1, 1, 1>, k_rpass<3, 1, 1, 1>},
            {nullptr, k_rpass<1, 1, 1, 2>, k_rpass<2, 1, 1, 2>, k_rpass<3, 1, 1, 2>},
            {nullptr, k_rpass<1, 1, 1, 3>, k_rpass<2, 1, 1, 3>, k_rpass<3, 1, 1, 3>},
            {nullptr, k_rpass<1, 1, 1, 4>, k_rpass<2, 1, 1, 4>, k_rpass<3, 1, 1, 4>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 1, 1, 6>, k_rpass<2, 1, 1, 6>, k_rpass<3, 1, 1, 6>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 1, 1, 10>, k_rpass<2, 1, 1, 10>, k_rpass<3, 1, 1, 10>},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, nullptr, nullptr, nullptr},
            {nullptr, k_rpass<1, 1, 1, 14>, k_rpass<2, 1, 1, 14>, k_rpass<3, 1, 1, 14>},
            {nullptr, nullptr, nullptr, nullptr},
        },
    };
    if (logg < 1 || logg > 3 || dir < 0 || dir > 1 || mode < 0 || mode > 15) return nullptr;
    return tab[dir][mode][logg];
}

rp_fn rp_get_p2(int logg, int dir, int mode);
rp_fn rp_get_p4(int logg, int dir, int mode);

rp_fn rp_get(int l, int logg, int dir, int mode)
{
    switch (l) {
    case 1024: return rp_get_p1(logg, dir, mode);
    case 2048: return rp_get_p2(logg, dir, mode);
    case 4096: return rp_get_p4(logg, dir, mode);
    }
    return nullptr;
}

rp_pair_fn rp_chain_get_p1(int nb)
{
    static const rp_pair_fn tab[4] = {nullptr, k_rchain<1, 1>, k_rchain<1, 2>, k_rchain<1, 3>};
    return nb >= 1 && nb <= 3 ? tab[nb] : nullptr;
}

rp_pair_fn rp_pair_get_p1(int op)
{
    static const rp_pair_fn tab[6] = {k_rpair<1, OP_DOUBLE>, k_rpair<1, OP_HALFADD>, k_rpair<1, OP_FILL>,
                                      k_rpair<1, OP_FIX>, k_rpair<1, OP_TWOXMY>, k_rpair<1, OP_IBFLY>};
    return op >= 0 && op < 6 ? tab[op] : nullptr;
}

rp_pair_fn rp_pair_get_p2(int op);
rp_pair_fn rp_pair_get_p4(int op);
rp_pair_fn rp_chain_get_p2(int nb);
rp_pair_fn rp_chain_get_p4(int nb);

rp_pair_fn rp_chain_get(int l, int nb)
{
    switch (l) {
    case 1024: return rp_chain_get_p1(nb);
    case 2048: return rp_chain_get_p2(nb);
    case 4096: return rp_chain_get_p4(nb);
    }
    return nullptr;
}

rp_pair_fn rp_pair_get(int l, int op)
{
    switch (l) {
    case 1024: return rp_pair_get_p1(op);
    case 2048: return rp_pair_get_p2(op);
    case 4096: return rp_pair_get_p4(op);
    }
    return nullptr;
}

void (*rp_scale_get_p1(int nt))(u64 *, u64 *, int *, u32, u32, u32, u32, u32)
{
    return nt == 256 ? k_rscale<1, 256> : k_rscale<1>;
}

void (*rp_scale_get_p2(int nt))(u64 *, u64 *, int *, u32, u32, u32, u32, u32);
void (*rp_scale_get_p4(int nt))(u64 *, u64 *, int *, u32, u32, u32, u32, u32);

rp_scale_fn rp_scale_get(int l, int nt)
{
    switch (l) {
    case 1024: return rp_scale_get_p1(nt);
    case 2048: return rp_scale_get_p2(nt);
    case 4096: return rp_scale_get_p4(nt);
    }
    return nullptr;
}
