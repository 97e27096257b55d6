// rdispatch.hpp -- host-side view of the register-resident big-coefficient passes
// (rkernels.hpp, rpass_p*.hip)
#pragma once
#include <stddef.h>
#include <stdint.h>

struct PassArgs;
struct PairArgs;
typedef void (*rp_fn)(PassArgs);
typedef void (*rp_pair_fn)(PairArgs);

#define RP_NT 512   // threads per workgroup; two workgroups share a CU

// k_rpass at l = 4096 with three levels (G = 8: 256 KiB of coefficients per group) runs
// 1024 threads, one workgroup per CU: every thread still holds 16 limb pairs (80 VGPRs)
// likewise the four-level inverse passes at l = 2048 (16 coefficients, one limb pair each)
// and the three-level inverse passes at l = 2048 (half the limb pairs per thread: their
// 512-thread form spilled 70-130 B of registers)
#ifdef MPFFT_FWD1K
#define RP_FWD1K 1
#else
#define RP_FWD1K 0
#endif
constexpr int rp_nt(int l, int logg, int dir = 0)
{
    return (l == 4096 && logg == 3) || (l == 2048 && logg == 4) || (l == 2048 && logg == 3 && (dir == 1 || RP_FWD1K)) ? 1024 : RP_NT;
}
// limb pairs per thread and coefficient (thread t owns pairs t + NT r)
constexpr int rp_r(int PP, int NT) { return 512 * PP / NT; }

// k_rpass<LOGG, PP, DIR, MODE> for coefficients of l = 1024 PP limbs (PP = 1, 2, 4);
// MODE: DIR 0: 1 = MFA twiddle applied on load, 2 = split fused into the load, 3 = inputs
//               owe an earlier pass's pending exponents (PassArgs::pcarry);
//       DIR 1: bit 0 = general final multipliers (inverse twiddle, scaling), bit 1 = the
//               pass holds the transform's last level.
rp_fn rp_get(int l, int logg, int dir, int mode);

// most levels per pass: 32 limbs per thread (G l <= 16384 limbs per 512-thread workgroup,
// 32768 at l = 4096 with 1024 threads)
inline int rp_maxlogg(int l) { return l == 1024 ? 3 : l == 2048 ? 3 : l == 4096 ? 3 : 0; }   // l = 1024: G = 16 spills
// forward passes of four levels at l = 2048 (1024 threads, one workgroup per CU): built, and
// taken by the plans whose MFA split make_plan chooses for them
inline int rp_maxlogg_fwd4(int l) { return l == 2048 ? 4 : rp_maxlogg(l); }
inline int rp_maxlogg_dit(int l) { return l == 2048 ? 4 : rp_maxlogg(l); }

// LDS: NX exchange slots of 9 l bytes (limbs + 16-bit pair overflows) and the exponent
// table.  <= 73 984 B, so two workgroups fit in 160 KiB (l = 4096, G = 8: 147 600 B, one).
inline size_t rp_lds(int l, int logg)
{
    const int G = 1 << logg, NX = G / 2 > 2 ? G / 2 : 2;
    const int nt = rp_nt(l, logg, 0), R = 512 * (l / 1024) / nt;
    return (size_t)NX * 9 * l + 4 * (size_t)(3 * G + (G / 2) * logg)   // + exponent and slot tables
           + 20 * (size_t)(nt / 64) * G * R;                            // + rp_shift_all's edge table
}

// k_rpair<PP, OP>: the truncated inverse's pair steps (OP_DOUBLE .. OP_IBFLY, kernels.hpp)
rp_pair_fn rp_pair_get(int l, int op);
inline size_t rp_pair_lds(int l) { return (size_t)9 * l + 16; }

// k_rchain<PP, NB>: NB = 1..3 TWOXMY steps and the enclosing IBFLY in one launch (Exec::chain)
rp_pair_fn rp_chain_get(int l, int nb);
inline size_t rp_chain_lds(int l) { return (size_t)9 * l + 32; }

// k_rscale<PP>: x <- 2^e x, canonical (the 2^-(depth+1) scaling before the combine)
typedef void (*rp_scale_fn)(uint64_t *, uint64_t *, int *, unsigned, unsigned, unsigned, unsigned, unsigned);
rp_scale_fn rp_scale_get(int l, int nt = 512);   // nt: threads per workgroup (512 or 256)
inline size_t rp_scale_lds(int l) { return (size_t)9 * l + (size_t)l + 128; }   // slot + pair overflows + canon scratch
// threads per k_rscale workgroup (diagnostic A/B: MPFFT_SCALE_NT=256)
