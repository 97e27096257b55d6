/*
 * mpfft.h -- C ABI of the MI355X-native Schoenhage-Strassen multiplier
 * (libmpfft.so, built from mpir-fft_amd/csrc/ by __graft_entry__.build()).
 *
 * The drop-in entry point is new_mpn_mul, with exactly the reference's
 * signature and meaning:
 *     /root/reference/mul_fft.c:3190-3191
 *     void new_mpn_mul(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1,
 *                      mp_limb_t *i2, mp_size_t n2,
 *                      mp_bitcnt_t depth, mp_bitcnt_t w);
 * r1[0 .. n1+n2) = i1[0 .. n1) * i2[0 .. n2), little-endian 64-bit limbs,
 * convolution length 2^(depth+1) over Z/(2^(2^depth w) + 1).  The reference
 * checks nothing and "will just segfault" on bad parameters
 * (mul_fft.c:3186-3188); this library validates them and aborts with a message
 * (new_mpn_mul) or returns a status (mpfft_mul_ex / mpfft_mul_device).
 * The result is the exact product, bit-identical to GMP/MPIR mpn_mul and to the
 * reference new_mpn_mul with its pointwise-row fix.
 */
#ifndef MPFFT_H
#define MPFFT_H

#include <stddef.h>
#include <stdint.h>

#if !defined(__GMP_H__) && !defined(__MPIR_H__) && !defined(MPFFT_HAVE_MP_TYPES)
/* GMP/MPIR LP64 types (mp_limb_t 64-bit unsigned, mp_size_t long, mp_bitcnt_t unsigned long) */
typedef uint64_t mp_limb_t;
typedef long mp_size_t;
typedef unsigned long mp_bitcnt_t;
#endif

#define MPFFT_VERSION 2

#define MPFFT_OK 0
#define MPFFT_EINVAL 1          /* n1, n2 < 1; depth outside [2, 30]; n*w not a multiple of 64 */
#define MPFFT_ETOOBIG 2         /* j1 + j2 - 1 > 2^(depth+1): product does not fit */
#define MPFFT_EUNSUPPORTED 3    /* coefficient size n*w/64 > 4096 limbs */
#define MPFFT_ENOMEM 4
#define MPFFT_EHIP 5
#define MPFFT_ENODEV 6

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces new_mpn_mul, mul_fft.c:3190-3265 (host pointers; H2D, device pipeline, D2H). */
void new_mpn_mul(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1, mp_limb_t *i2, mp_size_t n2,
                 mp_bitcnt_t depth, mp_bitcnt_t w);

/* Same as new_mpn_mul, returning MPFFT_* instead of aborting.  Host pointers.
 * Thread-safe: the calling thread's current HIP device (hipSetDevice) selects a
 * per-device context (stream + grow-only workspace); calls on one device serialise. */
int mpfft_mul_ex(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2,
                 unsigned long depth, unsigned long w);

/* (depth, w) chooser: the reference leaves them to its caller (mul_fft.c:3190-3191).
 * Picks the valid pair (power-of-two w, coefficients of <= 4096 limbs) with the least
 * predicted MI355X time (measured table, profiles/r02/chooser_sweep.json).
 * Returns MPFFT_OK, or MPFFT_ETOOBIG when no supported pair holds the product. */
int mpfft_choose(long n1, long n2, unsigned long *depth, unsigned long *w);

/* mpn_mul-style entry: r1 = i1 * i2 with (depth, w) from mpfft_choose (host pointers). */
int mpfft_mul_auto(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2);

/* Free the calling thread's device context buffers (re-allocated by the next call). */
int mpfft_release(void);

/* Device-resident multiply: all pointers are device memory, work is queued on
 * `stream` (a hipStream_t, NULL = default) and not synchronised.  d_ws must hold
 * mpfft_workspace_bytes(n1, n2, depth, w) bytes. */
int mpfft_mul_device(uint64_t *d_r, const uint64_t *d_i1, long n1, const uint64_t *d_i2, long n2,
                     unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream);

size_t mpfft_workspace_bytes(long n1, long n2, unsigned long depth, unsigned long w);

/* 0 if (n1, n2, depth, w) is a valid call, else the MPFFT_* reason. */
int mpfft_check_params(long n1, long n2, unsigned long depth, unsigned long w);

/* out[10] = n, l, NC (= sqrt, columns), j1, j2, trunc, bits1, NR (rows), threads/workgroup, limbs/thread
 * (mul_fft.c:3193-3203). */
int mpfft_plan_info(long n1, long n2, unsigned long depth, unsigned long w, long *out);

/* ---- sqrt2 front end: replaces new_mpn_mul6, mul_fft.c:3573-3668 ----------------------
 * A length-4n convolution mod 2^N + 1 (N = 2^depth w) through the 4n-th root of unity
 * sqrt2^w, sqrt2 = 2^(3N/4) - 2^(N/4): twice the transform length of new_mpn_mul at the
 * same coefficient size, bits1 = (N - depth - 1)/2 (:3578).  Any w with 64 | N (odd w is
 * where sqrt2 matters).  The reference needs trunc > 2n; here smaller products also work. */
void new_mpn_mul6(mp_limb_t *r1, mp_limb_t *i1, mp_size_t n1, mp_limb_t *i2, mp_size_t n2,
                  mp_bitcnt_t depth, mp_bitcnt_t w);
int mpfft_mul6_ex(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2,
                  unsigned long depth, unsigned long w);
int mpfft_mul6_device(uint64_t *d_r, const uint64_t *d_i1, long n1, const uint64_t *d_i2, long n2,
                      unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream);
size_t mpfft_workspace_bytes6(long n1, long n2, unsigned long depth, unsigned long w);
int mpfft_check_params6(long n1, long n2, unsigned long depth, unsigned long w);
/* out[10] as mpfft_plan_info, for new_mpn_mul6 (mul_fft.c:3575-3603) */
int mpfft_plan_info6(long n1, long n2, unsigned long depth, unsigned long w, long *out);

/* Byte offsets inside a single-GPU workspace (tests / multi-GPU driver):
 * out[8] = digA, topA, cbA, digB, topB, cbB, slots per operand, carry-mask words per slot. */
int mpfft_workspace_layout(long n1, long n2, unsigned long depth, unsigned long w, size_t *out);

/* One stage of the pipeline on a single-GPU workspace (stage-parity tests, multi-GPU driver). */
#define MPFFT_STAGE_FWD_COLUMNS 0   /* split + truncated column DIF, both operands   (mul_fft.c:2374-2390) */
#define MPFFT_STAGE_FWD_ROWS 1      /* MFA twiddle + row DIF, canonical out           (mul_fft.c:2392-2408) */
#define MPFFT_STAGE_POINTWISE 2     /* mpn_mulmod_2expp1 over the trunc live slots    (mul_fft.c:3244-3253) */
#define MPFFT_STAGE_INV_ROWS 3      /* row DIT + MFA un-twiddle                       (mul_fft.c:2942-2957) */
#define MPFFT_STAGE_INV_COLUMNS 4   /* truncated column inverse                       (mul_fft.c:2959-2977) */
#define MPFFT_STAGE_SCALE 5         /* divide by 2^(depth+1), normalise               (mul_fft.c:3256-3260) */
#define MPFFT_STAGE_COMBINE 6       /* FFT_combine_bits                               (mul_fft.c:3261-3262) */
#define MPFFT_NSTAGES 7
/* (tests) the folded path's combine: the workspace's coefficients as the inverse
 * columns leave them -- reduced form, 2^-(depth+1) already applied, the rows the truncated
 * inverse doubles not yet doubled -- into the product; MPFFT_EUNSUPPORTED on plans that do not
 * fold (mpfft_stage_kernels names k_combine_red for them) */
#define MPFFT_STAGE_FOLD_COMBINE 7
int mpfft_stage(int stage, const uint64_t *d_i1, const uint64_t *d_i2, uint64_t *d_r, long n1, long n2,
                unsigned long depth, unsigned long w, void *d_ws, size_t ws_bytes, void *stream);

/* ---- multi-GPU: one rank's share of a column-sharded multiply (mpir-fft_amd/sharded.py) ----
 * Column layout (column passes, ITFT, scale): slot = pos * ccount + (c - c0), NR * ccount slots.
 * Row layout (row passes, pointwise, combine): rows r0 .. r0+rcount of NC/ccb column blocks,
 *   slot = (c / ccb) * rcount * ccb + (p - r0) * ccb + c % ccb, rcount * NC slots.
 * Each slot: dig[l] limbs, cb[cb_words] carry masks, top int32. */
typedef struct mpfft_shard {
    long n1, n2;
    unsigned long depth, w;
    int c0, ccount;           /* columns of the column passes */
    int r0, rcount;           /* computed row positions of the row passes */
    int ccb;                  /* columns per block of the row layout (= NC / ranks) */
    uint64_t *col_dig[2], *col_cb[2];
    int *col_top[2];
    uint64_t *row_dig[2], *row_cb[2];
    int *row_top[2];
    long src_chunk;           /* 0: d_i1/d_i2 are the whole operands; else this rank's column
                                 slices: for each position p < T/NC, `src_chunk` limbs from
                                 limb floor((p NC + c0) bits1 / 64) on (sharded.py) */
    /* optional third row-layout array (NULL: none).  When set and mpfft_shard_row_fused()
     * says so, the row DIF's last level runs inside the pointwise, whose product lands here
     * (the caller then treats it as the row array of operand 0).  Added in MPFFT_VERSION 2:
     * callers must zero-initialise the whole struct (memset or `= {0}`), so code written for
     * the version-1 layout that sets only the older fields passes NULL here; a non-NULL
     * triple is always taken as a live array. */
    uint64_t *rowc_dig, *rowc_cb;
    int *rowc_top;
} mpfft_shard;

/* 1 if the sharded row stages fuse the last row DIF level into the pointwise for these
 * parameters and ccb columns per row block (the caller then supplies rowc_*), else 0. */
int mpfft_shard_row_fused(long n1, long n2, unsigned long depth, unsigned long w, int ccb);

#define MPFFT_SHARD_FWD_COLUMNS 0   /* split + column DIF of both operands (column layout) */
#define MPFFT_SHARD_FWD_ROWS 1      /* twiddle + row DIF of both operands (row layout), canonical */
#define MPFFT_SHARD_POINTWISE 2     /* row layout A <- A * B */
#define MPFFT_SHARD_INV_ROWS 3      /* row DIT + un-twiddle of A (row layout) */
#define MPFFT_SHARD_INV_COLUMNS 4   /* truncated column inverse + scale of A (column layout), canonical */
#define MPFFT_SHARD_FWD_COLUMNS_A 5 /* MPFFT_SHARD_FWD_COLUMNS for operand 1 only (clears the combine flags) */
#define MPFFT_SHARD_FWD_COLUMNS_B 6 /* ... for operand 2 only: with _A, lets operand 1's exchange overlap it */
#define MPFFT_SHARD_FWD_COLUMNS_OWN 7 /* MPFFT_SHARD_FWD_COLUMNS, but only rows [r0, r0 + rcount) of the
                                         column layout are computed (replicated forward columns: every
                                         rank runs every column block for its own rows) */
int mpfft_shard_stage(int stage, const mpfft_shard *sh, const uint64_t *d_i1, const uint64_t *d_i2, void *stream);
/* The row stages (FWD_ROWS, POINTWISE, INV_ROWS) on local rows [lo, hi) of the shard only, so a
 * driver can run the row phase in chunks and start exchange #2 of a finished chunk early. */
int mpfft_shard_stage_rows(int stage, const mpfft_shard *sh, int lo, int hi, void *stream);

/* Combine the canonical coefficients of a rank's column layout (after MPFFT_SHARD_INV_COLUMNS)
 * into its product stripes.  The product is cut into S = world * Tr stripes
 * (mpfft_shard_partition): stripe s owns coefficients [s C, (s+1) C) and product limbs
 * [ms[s], ms[s+1]) (mpfft_shard_stripes).  Rank g (= c0 / ccount) holds stripes s = j world + g,
 * j < Tr -- its column-layout rows -- and writes stripe j's limbs to d_r + j SL.
 * d_halo: the H coefficients before each of its stripes (l limbs each; stripe j's at
 * d_halo + j H l), moved there by the copies of mpfft_shard_halo_plan.
 * phase 0: every stripe with carry-in 0; d_sums[2 j], [2 j + 1] = (carry out, every limb
 *          all-ones) of stripe j.
 * phase 1: d_sums_all = the world ranks' d_sums in rank order (world * Tr * 2 ints, e.g. an
 *          all-gather): adds the carry from the stripes below to each of the rank's stripes.
 * Both phases are queued on `stream`; nothing synchronises with the host. */
size_t mpfft_shard_combine_tmp_bytes(long n1, long n2, unsigned long depth, unsigned long w, int world);
int mpfft_shard_combine(const mpfft_shard *sh, int phase, uint64_t *d_r, const uint64_t *d_halo, int *d_sums,
                        const int *d_sums_all, void *d_tmp, size_t tmp_bytes, void *stream);

/* ---- multi-GPU from one C process (north_star: "host code stays C") ----------
 * The same column-sharded multiply as mpir-fft_amd/sharded.py (one process per GPU over
 * RCCL), driven from one host thread over G devices: every rank's stages on its own device
 * stream, the two exchanges and the halo as peer copies over xGMI (hipMemcpyPeerAsync; peer
 * access enabled between distinct devices), ordered by events; the stripe carries on the device.
 * (Tested with every rank on one device; the cross-device copies have not run on separate GPUs.)
 *
 * Partition of one multiply over `world` ranks (a power of two dividing the plan's NC,
 * out[2] of mpfft_plan_info -- at l = 2048 in truncation case b that is 2^(floor(depth/2)+1),
 * not the reference's 2^floor(depth/2)):
 *   rows[world + 1]  row positions: rank d owns live rows [rows[d], rows[d+1])
 *   info[7]          C (columns per rank), chunk (operand slice limbs per row position),
 *                    H (halo coefficients per stripe), Tr (= trunc / NC), fused (1: the
 *                    pointwise takes the row DIF's last level(s), mpfft_shard_row_fused at
 *                    ccb = C), SL (product limbs per stripe at most: the d_r stride),
 *                    S (stripes = world Tr) */
int mpfft_shard_partition(long n1, long n2, unsigned long depth, unsigned long w, int world,
                          long *rows, long *info);
/* ms[0 .. S] = the first product limb of each stripe (ms[S] = n1 + n2); returns S + 1, or
 * -MPFFT_* (cap: ms's capacity; ms == NULL: counted only). */
long mpfft_shard_stripes(long n1, long n2, unsigned long depth, unsigned long w, int world, long *ms, long cap);

/* One exchange as element copies between the ranks' arrays (column layout: NR*C slots per
 * operand; row layout: (rows[d+1]-rows[d])*NC slots), fields dig (l u64 per slot), cb
 * (cb_words u64 per slot), top (one int32 per slot). */
typedef struct mpfft_copy {
    int src, dst;              /* ranks */
    int op;                    /* operand 0 or 1 */
    int field;                 /* 0 dig, 1 cb, 2 top */
    int src_layout, dst_layout;    /* 0 column layout, 1 row layout */
    long src_off, dst_off, count;  /* in elements of the field */
} mpfft_copy;
#define MPFFT_XCHG_COL_TO_ROW 1   /* #1 after the forward columns: both operands, every field */
#define MPFFT_XCHG_ROW_TO_COL 2   /* #2 after the inverse rows: operand 0, every field */
#define MPFFT_LAYOUT_HALO 2       /* mpfft_copy.dst_layout of a halo copy: the receiver's d_halo */
/* Number of copies written to out (out == NULL: counted only; cap: out's capacity),
 * or -MPFFT_* on error. */
long mpfft_shard_exchange_plan(long n1, long n2, unsigned long depth, unsigned long w, int world, int which,
                               mpfft_copy *out, long cap);
/* The halo copies before the combine: for every stripe, the H coefficients before it, from
 * the column layout (canonical limbs, field 0) of the ranks holding them to the d_halo of
 * mpfft_shard_combine (dst_layout MPFFT_LAYOUT_HALO); offsets and counts in limbs.  At most a
 * few coefficients per stripe: this replaces moving the whole product to row owners. */
long mpfft_shard_halo_plan(long n1, long n2, unsigned long depth, unsigned long w, int world,
                           mpfft_copy *out, long cap);

/* r1 = i1 * i2 (host pointers) sharded over ngpus devices: devices[g] is rank g's HIP device
 * (NULL: 0 .. ngpus-1; a device may repeat -- ranks sharing one GPU, as the tests do).
 * ngpus must be a power of two dividing the plan's NC (mpfft_shard_partition).  Device
 * buffers are cached per device list (grow-only; mpfft_multi_release frees them).  Not
 * reentrant with itself: concurrent calls serialise on one lock. */
int mpfft_mul_multi(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2,
                    unsigned long depth, unsigned long w, int ngpus, const int *devices);

/* The operand slices rank `rank` of `world` reads (the device-resident entry's inputs):
 * mpfft_shard_src_limbs limbs per operand -- for each live row position q, `chunk` limbs from
 * limb floor((q NC + c0) bits1 / 64) on, of the rank's own column block, or of every block
 * in turn when the forward columns are replicated (two ranks; MPFFT_REPLICATE_COLUMNS). */
long mpfft_shard_src_limbs(long n1, long n2, unsigned long depth, unsigned long w, int world);
int mpfft_shard_pack(long n1, long n2, unsigned long depth, unsigned long w, int world, int rank,
                     const uint64_t *a, long na, uint64_t *out);

/* Device-resident multi-GPU multiply: d_src1[g], d_src2[g] are rank g's packed operand slices
 * (mpfft_shard_pack) in devices[g]'s memory; rank g's product stripes land in d_r[g]
 * (stripe j -- product limbs [ms[j world + g], ms[j world + g + 1]) -- at d_r[g] + j SL, Tr SL
 * limbs).  streams[g] (hipStream_t on devices[g]): the work starts after what is queued there
 * and is queued back onto it (nothing waits on the host); streams == NULL: the call returns
 * when the product is complete. */
int mpfft_mul_multi_device(long n1, long n2, unsigned long depth, unsigned long w, int ngpus, const int *devices,
                           const uint64_t *const *d_src1, const uint64_t *const *d_src2, uint64_t *const *d_r,
                           void *const *streams);
int mpfft_multi_release(void);
/* The event graph of `calls` back-to-back mpfft_mul_multi_device calls over `world` ranks, as
 * text (no GPU touched, nothing allocated): one line per cross-stream ordering and per queued
 * piece of work -- "R d S ev" record, "W d S e ev" wait, "K d S what" rank-local work,
 * "C d S what e" a copy from rank e, "N" next call (multi.hip, the event graph).  Returns the
 * bytes needed including the terminating 0 (buf may be null), or a negative MPFFT_E* code. */
long mpfft_multi_schedule(long n1, long n2, unsigned long depth, unsigned long w, int world, int calls, char *buf,
                          size_t len);

/* new_mpn_mul / mpfft_mul_ex policy: with ngpus > 1 devices set, products whose coefficients
 * have >= min_l limbs (0: 1024) and whose NC the device count divides run through
 * mpfft_mul_multi; everything else on the calling thread's device as before.  ngpus <= 1
 * turns it off.  The environment variable MPFFT_DEVICES="0,1,...,7" (read at the first
 * multiply) sets the same policy for callers that cannot call this (an unmodified MPIR). */
int mpfft_set_devices(int ngpus, const int *devices, long min_l);
/* Devices the calling thread's last mpfft_mul_ex / new_mpn_mul ran on (1: single device). */
int mpfft_last_ngpus(void);

/* Stage profiling of the whole-multiply entries (new_mpn_mul, mpfft_mul_ex,
 * mpfft_mul_device): between begin and end, each of the next max_calls multiplies
 * records a HIP event on its own stream at every stage boundary (no other change to
 * the work); end synchronises and returns the summed per-stage milliseconds
 * (stage_ms[MPFFT_NSTAGES], MPFFT_STAGE_* order) and the number of profiled calls. */
int mpfft_profile_begin(int max_calls);
/* The kernel that carries each stage for these parameters, ';'-separated in MPFFT_STAGE_* order. */
int mpfft_stage_kernels(long n1, long n2, unsigned long depth, unsigned long w, char *buf, size_t len);
int mpfft_profile_end(float *stage_ms, int *calls);

const char *mpfft_strerror(int code);
int mpfft_version(void);

/* splitmix64-seeded xoshiro256** limbs (the benchmark's synthetic operands). */
void mpfft_fill_random(uint64_t *buf, long cnt, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif /* MPFFT_H */
