// pkernels.hpp -- sub-quadratic pointwise products mod p = 2^N + 1 for big coefficients
// (the nested negacyclic transform of FFT_mulmod_2expp1 /
// fft_mulmod_2expp1, mul_fft.c:2998-3167, FFT/IFFT_radix2_negacyclic :1290, :1861).
//
// One workgroup computes one product a b mod p (a, b canonical, N = 64 l bits):
//   * a, b are cut into K = 2^lk pieces of B = N/K bits (thread t owns piece t);
//   * the negacyclic convolution of the pieces (X^K == -1 with X = 2^B, so it IS the
//     product mod p) is computed in the inner ring R' = Z/(2^N' + 1), N' = 64 M, with
//     N' >= 2B + lk + 2 so every signed convolution coefficient |c_t| < K 2^(2B) is
//     recovered exactly from its residue (the reference instead restores the top
//     with a naive convolution of the low limbs, :3088; headroom is cheaper here);
//   * negacyclic weights theta^t = 2^(t N'/K), then a length-K cyclic DIF transform
//     with root omega = theta^2, pointwise products in R', DIT inverse, division by
//     K and un-weighting -- all multiplications by powers of two.
// Thread t holds its coefficient (M limbs + a small signed top word, value =
// limbs + top 2^N') in registers: additions are in-thread carry chains
// (v_add_co / v_addc).  A butterfly partner is read from LDS (limb-major,
// conflict-free) already rotated by the relative exponent; each thread keeps a
// *pending* exponent so its own value is never rotated.  The inner products are
// in-thread product-scanning schoolbook on 32-bit digits (v_mad_u64_u32).
// The coefficients are then summed (with their signs and the negacyclic wrap) into
// the l output limbs and stored in the reduced HBM form the inverse pass loads.
#pragma once
#include "coeff.hpp"

// LDS of one k_pwss workgroup: (M + 1) K limbs + tops + pending exponents + l overflows
__host__ __device__ constexpr size_t pw_lds_bytes(int M, int K, int l)
{
    return (size_t)(M + 1) * K * 8 + (size_t)K * 8 + (size_t)l * 4;
}

// r = alpha * own + 2^E * x_q  (mod p', not reduced); alpha in {-1, 0, 1}.
// x_q: limbs X[i K + q], top TT[q].  Derivation (E' = E mod N' = 64 Y + s):
//   2^(64 Y) x == W + 1 - (1 + T) 2^(64 Y),  W_j = X_(j-Y) (j >= Y), ~X_(j-Y+M) (j < Y)
//   2^s W == U - ov,  U = W << s (M limbs), ov = the s bits shifted out of the top
//   2^E' x == U + (2^s - ov) - (1 + T) 2^(64 Y + s);  E >= N' negates (2^N' == -1).
template <int M>
__host__ __device__ __forceinline__ void pw_combine(u64 (&L)[M], int &T, int alpha, const u64 *X, const int *TT, int K,
                                                   int q, unsigned E)
{
    constexpr unsigned NP = 64 * M;
    const bool neg = E >= NP;   // 2^N' == -1: subtract instead
    if (neg) E -= NP;
    const int Y = (int)(E >> 6), s = (int)(E & 63);
    const i64 Tq = TT[q];
    i64 c = 0;                  // signed carry into the next limb
    if (alpha < 0) {            // -(L + T 2^N') = ~L + 1 + (-1 - T) 2^N'
#pragma unroll
        for (int j = 0; j < M; ++j) L[j] = ~L[j];
        c = 1;
        T = -1 - T;
    } else if (alpha == 0) {
#pragma unroll
        for (int j = 0; j < M; ++j) L[j] = 0;
        T = 0;
    }
    // U = (W << s) + C0 at limb 0 + CY at limb Y (128-bit signed corrections, lo + hi 2^64)
    const u64 wtop = X[(M - 1 - Y) * K + q];                  // W_(M-1), never wrapped (Y < M)
    const u64 ov = (wtop >> 1) >> (63 - s);                   // the s bits shifted out (s == 0: 0)
    u64 c0lo = ((u64)1 << s) - ov;                            // 2^s - ov in (0, 2^63]
    i64 c0hi = 0;
    const i64 v = -(1 + Tq);
    u64 cylo = (u64)v << s;                                   // (1 + T) 2^s, negated
    i64 cyhi = (v >> 1) >> (63 - s);
    if (Y == 0) {   // both corrections at limb 0
        const u64 t = c0lo + cylo;
        c0hi += cyhi + (i64)(t < c0lo);
        c0lo = t;
        cylo = 0;
        cyhi = 0;
    }
    u64 smask = 0;
    if (neg) {      // -U = ~U + 1 - 2^N', corrections negated
        smask = ~(u64)0;
        c += 1;
        T -= 1;
        c0hi = -c0hi - (i64)(c0lo != 0);
        c0lo = (u64)0 - c0lo;
        cyhi = -cyhi - (i64)(cylo != 0);
        cylo = (u64)0 - cylo;
    }
    u64 wprev = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        int src = j - Y;
        const bool wr = src < 0;
        src += wr ? M : 0;
        u64 w = X[src * K + q];
        w = wr ? ~w : w;
        const u64 x = ((w << s) | ((wprev >> 1) >> (63 - s))) ^ smask;
        wprev = w;
        // L_j + x + c + correction, carry kept signed (|c| <= 4)
        u64 r = L[j] + x;
        i64 cy = (i64)(r < x);
        const u64 r2 = r + (u64)c;
        cy += c >= 0 ? (i64)(r2 < r) : -(i64)(r2 > r);
        u64 cl = 0;
        i64 ch = 0;
        if (j == 0) { cl = c0lo; ch = c0hi; }
        if (j == Y && j != 0) { cl = cylo; ch = cyhi; }
        const u64 r3 = r2 + cl;
        cy += (i64)(r3 < r2) + ch;
        L[j] = r3;
        c = cy;
    }
    T += (int)c;
}

// canonical residue of L + T 2^N' (== L - T): limbs in [0, 2^N'), returns 1 for 2^N' (L = 0)
template <int M>
__host__ __device__ __forceinline__ int pw_canon(u64 (&L)[M], int T)
{
    i128 acc = -(i128)T;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        acc += (i128)L[j];
        L[j] = (u64)acc;
        acc >>= 64;
    }
    const int c1 = (int)(i64)acc;   // value == L - c1 now, |c1| <= 1
    acc = -(i128)c1;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        acc += (i128)L[j];
        L[j] = (u64)acc;
        acc >>= 64;
    }
    if ((i64)acc != 0) {   // the second fold wrapped: the value is 2^N' == -1
#pragma unroll
        for (int j = 0; j < M; ++j) L[j] = 0;
        return 1;
    }
    return 0;
}

// z = a b mod p' for canonical a (La, ta), b (Lb, tb); result limbs + top (value = L + T 2^N')
template <int M>
__host__ __device__ __forceinline__ void pw_mulmod(u64 (&Z)[M], int &T, const u64 (&La)[M], int ta, const u64 (&Lb)[M],
                                          int tb)
{
    if (ta | tb) {   // 2^N' == -1: the product is 1, -b or -a  (cf. mul_fft.c:3250)
        if (ta && tb) {
#pragma unroll
            for (int j = 0; j < M; ++j) Z[j] = j == 0;
            T = 0;
            return;
        }
        // -v = ~v + 1 - 2^N'  ->  limbs ~v, +1 at limb 0, top -1
#pragma unroll
        for (int j = 0; j < M; ++j) Z[j] = ta ? Lb[j] : La[j];
        i128 acc = 1;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            acc += (i128)(~Z[j]);
            Z[j] = (u64)acc;
            acc >>= 64;
        }
        T = -1 + (int)(i64)acc;
        return;
    }
    // Full product over 29-bit digits: a column sums at most ND < 64 products < 2^58,
    // so one v_mad_u64_u32 per digit product with no carry tracking.  Columns are
    // streamed into 64-bit limbs and folded on the fly: Z = lo - hi (2^N' == -1).
    constexpr int DB = 29, ND = (64 * M + DB - 1) / DB;
    static_assert(ND < 64, "column sums must stay below 2^64");
    u32 ad[ND], bd[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const int b0 = d * DB, li = b0 >> 6, sh = b0 & 63;
        u64 x = La[li] >> sh, y = Lb[li] >> sh;
        if (sh + DB > 64 && li + 1 < M) {
            x |= La[li + 1] << (64 - sh);
            y |= Lb[li + 1] << (64 - sh);
        }
        ad[d] = (u32)(x & ((1u << DB) - 1));
        bd[d] = (u32)(y & ((1u << DB) - 1));
    }
    u128 acc = 0;          // bits [pos, ...) of the product not yet emitted
    int pos = 0, k = 0;    // compile-time after unrolling
    i64 bw = 0;            // borrow of the lo - hi fold
#pragma clang loop unroll(full)
    for (int c = 0; c < 2 * ND - 1; ++c) {
        u64 col = 0;
        const int i0 = c < ND ? 0 : c - ND + 1, i1 = c < ND ? c : ND - 1;
#pragma clang loop unroll(full)
        for (int i = i0; i <= i1; ++i) col += (u64)ad[i] * bd[c - i];
        acc += (u128)col << (DB * c - pos);
        const bool last = c == 2 * ND - 2;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            if (k < 2 * M && (last || DB * (c + 1) - pos >= 64)) {
                const u64 limb = (u64)acc;
                acc >>= 64;
                pos += 64;
                if (k < M) {
                    Z[k] = limb;
                } else {                       // fold: Z[k - M] -= limb (borrow chain)
                    const u64 z = Z[k - M];
                    const u64 d1 = z - limb;
                    i64 b1 = (i64)(d1 > z);
                    const u64 d2 = d1 + (u64)bw;   // bw <= 0
                    b1 += bw < 0 ? (i64)(d2 > d1) : 0;
                    Z[k - M] = d2;
                    bw = -b1;
                }
                ++k;
            }
        }
    }
    T = (int)bw;   // value = Z + T 2^N', T in {-1, 0}
}

// exchange: thread t publishes its value (limbs L, top T) in the limb-major LDS buffer
template <int M>
__device__ __forceinline__ void pw_publish(const u64 (&L)[M], int T, u64 *X, int *TT, int K, int t)
{
#pragma unroll
    for (int j = 0; j < M; ++j) X[j * K + t] = L[j];
    TT[t] = T;
}

// One forward (DIF) or inverse (DIT) length-K cyclic transform with root 2^(2 TH) over
// the values of the K threads of this workgroup.  P: this thread's pending exponent.
template <int M, int DIR>
__device__ __forceinline__ void pw_transform(u64 (&L)[M], int &T, unsigned &P, u64 *X, int *TT, unsigned *PP, int lk,
                                             unsigned TH, int t)
{
    const int K = 1 << lk;
    constexpr unsigned N2 = 128 * M;
    for (int jj = 0; jj < lk; ++jj) {
        const int j = DIR == 0 ? jj : lk - 1 - jj;   // DIF level index (DIT runs them backwards)
        const int h = K >> (j + 1);
        const int q = t ^ h;
        const bool top = !(t & h);
        const int qt = t & ~h;                       // top index of the pair
        const unsigned tw = (unsigned)(((u64)(qt & (h - 1)) << j) * (2 * TH) % N2);
        pw_publish<M>(L, T, X, TT, K, t);
        PP[t] = P;
        __syncthreads();
        const unsigned Pq = PP[q];
        unsigned E;
        int alpha;
        if (DIR == 0) {
            // top: X_t + X_q = 2^P (x_t + 2^(Pq-P) x_q); bottom: (X_q - X_t) w^tw = 2^(P+tw) (2^(Pq-P) x_q - x_t)
            E = (Pq + N2 - P) % N2;
            alpha = top ? 1 : -1;
            pw_combine<M>(L, T, alpha, X, TT, K, q, E);
            if (!top) P = (P + tw) % N2;
        } else {
            // top: Z_t + Z_q w^-tw = 2^P (z_t + 2^(Pq-tw-P) z_q)
            // bottom: Z_q - Z_t w^-tw = 2^(P-tw) (2^(Pq-P+tw) z_q - z_t)
            E = top ? (Pq + 2 * N2 - tw - P) % N2 : (Pq + N2 - P + tw) % N2;
            alpha = top ? 1 : -1;
            pw_combine<M>(L, T, alpha, X, TT, K, q, E);
            if (!top) P = (P + N2 - tw) % N2;
        }
        __syncthreads();
    }
}

// k_pwss<M>: A[slot] <- A[slot] * B[slot] mod 2^N + 1, one workgroup of K = 2^lk threads
// per slot; canonical inputs (limbs + carry limb in {0, 1}), reduced-form output.
template <int M>
__global__ __launch_bounds__(512) void k_pwss(u64 *digA, u64 *cbA, int *topA, const u64 *digB, const int *topB, int l,
                                              int lk, unsigned long long *dbg)
{
    // diagnostics (MPFFT_PW_STAMPS): thread 0 stamps the phase boundaries of this workgroup
    unsigned long long *stamp = dbg ? dbg + 8 * (size_t)blockIdx.x : nullptr;
#define PW_STAMP(k) do { if (stamp && threadIdx.x == 0) stamp[k] = __builtin_amdgcn_s_memtime(); } while (0)
    PW_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int K = 1 << lk, t = threadIdx.x;
    const int LP = l >> lk;                      // limbs per piece
    constexpr unsigned NP = 64 * M, N2 = 2 * NP;
    const unsigned TH = NP >> lk;                // theta = 2^TH
    u64 *X = (u64 *)smem;                        // (M + 1) K limbs
    int *TT = (int *)(X + (size_t)(M + 1) * K);  // K
    unsigned *PP = (unsigned *)(TT + K);         // K
    int *H = (int *)(PP + K);                    // l
    const long slot = blockIdx.x;
    const int ta = topA[slot], tb = topB[slot];
    u64 *pa = digA + (size_t)slot * l;
    const u64 *pb = digB + (size_t)slot * l;
    const int lane = t & 63;
    const int cbw = cb_words(l);
    u64 *cbp = cbA + (size_t)slot * cbw;

    if (ta | tb) {
        // 2^N == -1: the product is 1, -b or -a (mul_fft.c:3250).  -v == ~v + 2 (mod p):
        // limbs ~v with the +2 carried by the carry limb (top = -2, weighs 2^N == -1).
        for (int m = t; m < l; m += K) {
            const u64 v = ta && tb ? (m == 0) : ~(ta ? pb[m] : pa[m]);
            pa[m] = v;
        }
        for (int w = t; w < cbw; w += K) cbp[w] = 0;
        if (t == 0) topA[slot] = ta && tb ? 0 : -2;
        return;
    }

    // ---- pieces and forward transforms (A, then B held in registers) -----------------
    u64 La[M], Lb[M];
    int Ta = 0, Tb = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        La[j] = j < LP ? pa[(size_t)t * LP + j] : 0;
        Lb[j] = j < LP ? pb[(size_t)t * LP + j] : 0;
    }
    unsigned Pa = (unsigned)(((u64)t * TH) % N2), Pb = Pa;   // negacyclic weight theta^t
    PW_STAMP(1);
    pw_transform<M, 0>(La, Ta, Pa, X, TT, PP, lk, TH, t);
    PW_STAMP(2);
    pw_transform<M, 0>(Lb, Tb, Pb, X, TT, PP, lk, TH, t);
    PW_STAMP(3);

    // ---- inner products: 2^Pa xa * 2^Pb xb = 2^(Pa + Pb) (xa xb) ---------------------
    const int ca = pw_canon<M>(La, Ta), cb = pw_canon<M>(Lb, Tb);
    u64 Z[M];
    int Tz;
    pw_mulmod<M>(Z, Tz, La, ca, Lb, cb);
    unsigned Pz = (Pa + Pb) % N2;
    PW_STAMP(4);

    // ---- inverse, then 2^-lk (division by K) and theta^-t --------------------------
    pw_transform<M, 1>(Z, Tz, Pz, X, TT, PP, lk, TH, t);
    PW_STAMP(5);
    {
        const unsigned un = (unsigned)(((u64)t * TH + lk) % N2);
        const unsigned F = (Pz + N2 - un) % N2;
        pw_publish<M>(Z, Tz, X, TT, K, t);
        __syncthreads();
        pw_combine<M>(Z, Tz, 0, X, TT, K, t, F);
        __syncthreads();
    }
    // signed coefficient c_t = v - s p', v in [0, 2^N'], s = (v > 2^(N'-1))
    const int zt = pw_canon<M>(Z, Tz);
    const int neg = zt || (Z[M - 1] >> 63);
#pragma unroll
    for (int j = 0; j < M; ++j) X[j * K + t] = Z[j];
    X[(size_t)M * K + t] = (u64)zt;              // limb M of v (2^N' only)
    TT[t] = neg;
    __syncthreads();
    PW_STAMP(6);

    // ---- combine: R = sum_t c_t 2^(B t) mod 2^N + 1 -------------------------------------
    // c_t 2^(Bt) = v_t 2^(Bt) - s_t (2^(Bt) + 2^(N' + Bt)); positions >= N wrap negated.
    // Thread t sums output limbs m = t + K r (coalesced, consecutive per wave).
    u64 fo[8];
    int ho[8];
    const int RPT = l / K;   // <= 8 (host)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        fo[r] = 0;
        ho[r] = 0;
        if (r >= RPT) continue;
        const int m = t + K * r;
        i128 S = 0;
        // pieces whose limbs [t'LP, t'LP + M] cover m, directly and through the wrap (m + l)
#pragma unroll
        for (int wrap = 0; wrap < 2; ++wrap) {
            const int mm = m + wrap * l;
            int lo = (mm - M + LP - 1) / LP;       // ceil((mm - M) / LP) for mm >= M
            if (mm < M) lo = 0;
            int hi = mm / LP;
            if (hi > K - 1) hi = K - 1;
            for (int tp = lo; tp <= hi; ++tp) {
                const int d = mm - tp * LP;        // limb of c_tp, 0 .. M
                i128 v = (i128)X[(size_t)d * K + tp];
                if (TT[tp] && (d == 0 || d == M)) v -= 1;
                S += wrap ? -v : v;
            }
        }
        fo[r] = (u64)S;
        ho[r] = (int)(i64)(S >> 64);
        H[m] = ho[r];
    }
    __syncthreads();
    // limb m: f_m + hv_(m-1) -> limb + carry out in {-1, 0, 1} (reduced form; the top
    // limb's overflow wraps into limb 0 negated, and its carry weighs 2^N == -1)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >= RPT) continue;
        const int m = t + K * r;
        const int hin = m ? H[m - 1] : -H[l - 1];
        const u64 f = fo[r];
        const u64 nf = f + (u64)(i64)hin;
        const int kout = hin >= 0 ? (int)(nf < f) : -(int)(nf > f);
        pa[m] = nf;
        const u64 pm = __ballot(kout == 1), nm = __ballot(kout == -1);
        if (lane == 0) {
            cbp[2 * (m >> 6)] = pm;
            cbp[2 * (m >> 6) + 1] = nm;
        }
    }
    if (t == 0) topA[slot] = 0;
    if (stamp) {
        __syncthreads();
        PW_STAMP(7);
    }
#undef PW_STAMP
}
