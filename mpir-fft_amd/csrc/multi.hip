// multi.hip -- the column-sharded multiply over G devices from one C process.
//
// The matrix Fourier algorithm's column transforms are independent per column
// (/root/reference/mul_fft.c:2374-2390), its row transforms, pointwise products and row
// inverses per row (:2392-2408, :3244-3253, :2942-2957), its column inverses per column
// (:2959-2977).  Rank g (device devices[g]) owns columns [g C, (g+1) C) and live rows
// [rows[g], rows[g+1]):
//
//   H2D       rank g's operand column slices (packed on the host, one thread per rank)
//   stage     split + forward column passes                   (mpfft_shard_stage)
//   xchg #1   column layout -> row layout, both operands      (peer copies over xGMI)
//             -- at two ranks both compute every column block instead (all blocks' slices
//             H2D) and keep their rows of each: exchange #1 becomes local copies
//   stage     forward rows, pointwise, inverse rows
//   xchg #2   row layout -> column layout, the product
//   stage     truncated inverse columns + scale
//   xchg #3   canonical coefficients -> contiguous ranges; H halo coefficients from rank g-1
//   combine   phase 0 (carry-in 0) per rank, the cross-rank carry on the host, phase 1
//   D2H       rank g's product limbs [M_g, M_g+1) (one thread per rank)
//
// Every rank's work is queued on its own stream; an exchange's copies run on the receiving
// rank's stream after it waited for the senders' events (pull), so no host barrier sits
// between stages and ranks sharing a device (the one-GPU tests) need nothing special.
// This is the same pipeline as mpir-fft_amd/sharded.py (one process per GPU, RCCL); the
// partition and the exchange plans are the C functions both use.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mpfft.h"

typedef uint64_t u64;

void mpfft_note_hip_error(hipError_t e);   // mpfft.c: what mpfft_strerror(MPFFT_EHIP) reports

namespace {

struct Part {
    int world;
    long n1, n2, total, n, l, NC, NR, T, Tr, bits1, N, len;
    long C, chunk, H, cbw;
    bool fused;
    bool rep;      // replicated forward columns: every rank computes every column block (world 2)
    long nsl() const { return rep ? world : 1; }   // operand column slices a rank holds
    std::vector<long> rows, M;
    long rcount(int d) const { return rows[d + 1] - rows[d]; }
};

long cb_words_l(long l) { return 2 * ((l + 63) / 64); }

// ShardPlan (sharded.py) in C: the same arithmetic, so both drivers agree slot for slot
int partition(Part &p, long n1, long n2, unsigned long depth, unsigned long w, int world)
{
    long info[10];
    int rc = mpfft_plan_info(n1, n2, depth, w, info);
    if (rc) return rc;
    p.world = world;
    p.n1 = n1;
    p.n2 = n2;
    p.total = n1 + n2;
    p.n = info[0];
    p.l = info[1];
    p.NC = info[2];
    p.T = info[5];
    p.bits1 = info[6];
    p.NR = info[7];
    p.len = info[3] + info[4] - 1;
    p.N = p.n * (long)w;
    p.Tr = p.T / p.NC;
    if (world < 1 || (world & (world - 1)) || p.NC % world) return MPFFT_EINVAL;
    p.C = p.NC / world;
    p.rows.assign(world + 1, 0);
    for (int d = 0; d <= world; ++d) p.rows[d] = ((long)d * p.Tr) / world;
    p.M.assign(world + 1, 0);
    for (int d = 1; d < world; ++d) {
        const long m = (long)(((unsigned __int128)(p.rows[d] * p.NC) * (u64)p.bits1) / 64);
        p.M[d] = m < p.total ? m : p.total;
    }
    p.M[world] = p.total;
    p.H = (p.N + 128 + p.bits1 - 1) / p.bits1 + 1;
    p.cbw = cb_words_l(p.l);
    for (int d = 1; d < world; ++d) {
        if (p.rows[d] * p.NC < p.H) return MPFFT_EINVAL;       // the halo would span ranks
        if (p.rows[d + 1] - p.rows[d] < 1) return MPFFT_EINVAL;  // a rank without rows
    }
    if (p.Tr < world) return MPFFT_EINVAL;
    p.chunk = (p.C * p.bits1 + 63) / 64 + 2;
    p.fused = mpfft_shard_row_fused(n1, n2, depth, w, (int)p.C) != 0;
    p.rep = false;
    return MPFFT_OK;
}

long field_width(const Part &p, int f) { return f == 0 ? p.l : f == 1 ? p.cbw : 1; }

// the copies of one exchange (sharded.py ShardedMul._col_to_row / _row_to_col)
void exchange_plan(const Part &p, int which, std::vector<mpfft_copy> &out)
{
    out.clear();
    const int nf = which == MPFFT_XCHG_COEFFS ? 1 : 3;
    const int nop = which == MPFFT_XCHG_COL_TO_ROW ? 2 : 1;
    for (int d = 0; d < p.world; ++d)          // row-layout rank (receiver of #1/#3, sender of #2)
        for (int s = 0; s < p.world; ++s)      // column-layout rank
            for (int op = 0; op < nop; ++op)
                for (int f = 0; f < nf; ++f) {
                    const long wd = field_width(p, f);
                    const long cnt = p.rcount(d) * p.C * wd;
                    mpfft_copy c;
                    const long col_off = p.rows[d] * p.C * wd, row_off = (long)s * cnt;
                    if (which == MPFFT_XCHG_ROW_TO_COL) {
                        c = {d, s, op, f, 1, 0, row_off, col_off, cnt};
                    } else {
                        c = {s, d, op, f, 0, 1, col_off, row_off, cnt};
                    }
                    if (cnt) out.push_back(c);
                }
}

struct Arr {
    u64 *dig = nullptr, *cb = nullptr;
    int *top = nullptr;
};

struct Rank {
    int dev = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    hipStream_t xs = nullptr;    // exchange #1's copies (overlapping operand 2's column passes)
    hipEvent_t eva = nullptr;    // operand 1's column passes done
    hipEvent_t evx = nullptr;    // exchange #1 done
    unsigned char *mem = nullptr;
    size_t mem_bytes = 0;
    u64 *host = nullptr;      // pinned staging of the operand slices
    size_t host_bytes = 0;
    Arr col[2], row[2], colc, rowc;
    u64 *src[2] = {nullptr, nullptr};
    u64 *halo = nullptr, *r = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    int *sum = nullptr;
};

struct Ctx {
    std::mutex mu;
    std::vector<int> devs;
    std::vector<Rank> ranks;
};
Ctx g_ctx;

#define MCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { mpfft_note_hip_error(e_); return MPFFT_EHIP; } } while (0)

size_t al(size_t x) { return (x + 255) / 256 * 256; }

void free_rank(Rank &R)
{
    if (R.s) {
        (void)hipSetDevice(R.dev);
        (void)hipStreamSynchronize(R.s);
    }
    if (R.mem) (void)hipFree(R.mem);
    if (R.host) (void)hipHostFree(R.host);
    if (R.xs) (void)hipStreamSynchronize(R.xs);
    if (R.ev) (void)hipEventDestroy(R.ev);
    if (R.eva) (void)hipEventDestroy(R.eva);
    if (R.evx) (void)hipEventDestroy(R.evx);
    if (R.s) (void)hipStreamDestroy(R.s);
    if (R.xs) (void)hipStreamDestroy(R.xs);
    R = Rank();
}

// carve rank d's arrays out of one grow-only allocation
int setup_rank(const Part &p, int d, Rank &R)
{
    MCHK(hipSetDevice(R.dev));
    if (!R.s) MCHK(hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking));
    if (!R.ev) MCHK(hipEventCreateWithFlags(&R.ev, hipEventDisableTiming));
    if (!R.xs) MCHK(hipStreamCreateWithFlags(&R.xs, hipStreamNonBlocking));
    if (!R.eva) MCHK(hipEventCreateWithFlags(&R.eva, hipEventDisableTiming));
    if (!R.evx) MCHK(hipEventCreateWithFlags(&R.evx, hipEventDisableTiming));
    const long cs = p.NR * p.C, rs = p.rcount(d) * p.NC;
    const long mcount = p.M[d + 1] - p.M[d];
    const bool w1 = p.world == 1;
    const int ncol = (w1 && p.fused) ? 3 : 2;          // world 1: the fused product's column array
    const int nrow = w1 ? 0 : (p.fused ? 3 : 2);      // world 1: row arrays are views
    auto arr_bytes = [&](long slots) { return al(slots * p.l * 8) + al(slots * p.cbw * 8) + al(slots * 4); };
    const size_t tmpb = mpfft_shard_combine_tmp_bytes(mcount > 0 ? mcount : 1);
    const long sl = p.nsl() * p.Tr * p.chunk;        // operand slices held (all blocks' when replicated)
    const size_t need = ncol * arr_bytes(cs) + nrow * arr_bytes(rs) + 2 * al(sl * 8) +
                        al(p.H * p.l * 8) + al((mcount > 0 ? mcount : 1) * 8) + al(tmpb) + 256;
    if (R.mem_bytes < need) {
        if (R.mem) MCHK(hipFree(R.mem));
        R.mem = nullptr;
        R.mem_bytes = 0;
        if (hipMalloc((void **)&R.mem, need) != hipSuccess) return MPFFT_ENOMEM;
        R.mem_bytes = need;
        MCHK(hipMemsetAsync(R.mem, 0, need, R.s));   // zero carry masks / carry limbs, as sharded.py
    }
    unsigned char *q = R.mem;
    auto carve = [&](long slots) {
        Arr a;
        a.dig = (u64 *)q; q += al(slots * p.l * 8);
        a.cb = (u64 *)q; q += al(slots * p.cbw * 8);
        a.top = (int *)q; q += al(slots * 4);
        return a;
    };
    R.col[0] = carve(cs);
    R.col[1] = carve(cs);
    R.colc = ncol == 3 ? carve(cs) : Arr();
    if (w1) {   // one rank: the row layout (ccb = NC, rows [0, Tr)) is the column layout's first slots
        R.row[0] = R.col[0];
        R.row[1] = R.col[1];
        R.rowc = R.colc;
    } else {
        R.row[0] = carve(rs);
        R.row[1] = carve(rs);
        R.rowc = p.fused ? carve(rs) : Arr();
    }
    R.src[0] = (u64 *)q; q += al(sl * 8);
    R.src[1] = (u64 *)q; q += al(sl * 8);
    R.halo = (u64 *)q; q += al(p.H * p.l * 8);
    R.r = (u64 *)q; q += al((mcount > 0 ? mcount : 1) * 8);
    R.tmp = q; q += al(tmpb);
    R.tmp_bytes = tmpb;
    R.sum = (int *)q;
    const size_t hb = (size_t)2 * sl * 8;
    if (R.host_bytes < hb) {
        if (R.host) MCHK(hipHostFree(R.host));
        R.host = nullptr;
        R.host_bytes = 0;
        if (hipHostMalloc((void **)&R.host, hb, hipHostMallocDefault) != hipSuccess) return MPFFT_ENOMEM;
        R.host_bytes = hb;
    }
    return MPFFT_OK;
}

mpfft_shard desc(const Part &p, int d, const Rank &R, unsigned long depth, unsigned long w)
{
    mpfft_shard sh;
    memset(&sh, 0, sizeof(sh));
    sh.n1 = p.n1;
    sh.n2 = p.n2;
    sh.depth = depth;
    sh.w = w;
    sh.c0 = (int)(d * p.C);
    sh.ccount = (int)p.C;
    sh.r0 = (int)p.rows[d];
    sh.rcount = (int)p.rcount(d);
    sh.ccb = (int)p.C;
    for (int k = 0; k < 2; ++k) {
        sh.col_dig[k] = R.col[k].dig;
        sh.col_cb[k] = R.col[k].cb;
        sh.col_top[k] = R.col[k].top;
        sh.row_dig[k] = R.row[k].dig;
        sh.row_cb[k] = R.row[k].cb;
        sh.row_top[k] = R.row[k].top;
    }
    sh.src_chunk = p.chunk;
    if (p.fused) {
        sh.rowc_dig = R.rowc.dig;
        sh.rowc_cb = R.rowc.cb;
        sh.rowc_top = R.rowc.top;
    }
    return sh;
}

// rank d's column slices of operand a: for each live row position q, `chunk` limbs from limb
// floor((q NC + d C) bits1 / 64) on (ShardPlan.slice_operand)
void pack_slice(const Part &p, int d, const u64 *a, long na, u64 *out)
{
    for (long q = 0; q < p.Tr; ++q) {
        u64 *o = out + q * p.chunk;
        const long s0 = (long)(((unsigned __int128)(q * p.NC + d * p.C) * (u64)p.bits1) / 64);
        long cnt = 0;
        if (s0 < na) {
            cnt = na - s0 < p.chunk ? na - s0 : p.chunk;
            memcpy(o, a + s0, (size_t)cnt * 8);
        }
        if (cnt < p.chunk) memset(o + cnt, 0, (size_t)(p.chunk - cnt) * 8);
    }
}

void *field_ptr(const Arr &a, int f, long off)
{
    if (f == 0) return a.dig + off;
    if (f == 1) return a.cb + off;
    return a.top + off;
}

// queue one copy of an exchange plan on stream `st` of its receiving rank
int queue_copy(const std::vector<Rank> &rk, const mpfft_copy &c, hipStream_t st)
{
    const Rank &S = rk[c.src], &D = rk[c.dst];
    const Arr &sa = c.src_layout ? S.row[c.op] : S.col[c.op];
    const Arr &da = c.dst_layout ? D.row[c.op] : D.col[c.op];
    const size_t es = c.field == 2 ? 4 : 8;
    void *dp = field_ptr(da, c.field, c.dst_off);
    const void *sp = field_ptr(sa, c.field, c.src_off);
    if (dp == sp) return MPFFT_OK;   // world 1: the row layout is a view of the column layout
    if (S.dev == D.dev) MCHK(hipMemcpyAsync(dp, sp, c.count * es, hipMemcpyDeviceToDevice, st));
    else MCHK(hipMemcpyPeerAsync(dp, D.dev, sp, S.dev, c.count * es, st));
    return MPFFT_OK;
}

// exchange #1 with the forward column passes run per operand: every receiver's exchange
// stream pulls operand 1's blocks once all senders finished operand 1's passes (event eva)
// -- while the compute streams run operand 2's passes -- then operand 2's (event ev); the
// compute stream waits for both before the row passes
int run_exchange_fwd(const Part &p, std::vector<Rank> &rk);

// replicated forward columns (world 2): rank d runs every column block e's split + column
// passes from block e's operand slices into its own column arrays (scratch), then plays
// exchange #1's copies from e to d locally -- its rows of block e into its row layout
int fwd_replicated(const Part &p, std::vector<Rank> &rk, unsigned long depth, unsigned long w)
{
    std::vector<mpfft_copy> plan;
    exchange_plan(p, MPFFT_XCHG_COL_TO_ROW, plan);
    const long sl = p.Tr * p.chunk;
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        MCHK(hipSetDevice(R.dev));
        for (int e = 0; e < p.world; ++e) {
            mpfft_shard sh = desc(p, d, R, depth, w);
            sh.c0 = (int)(e * p.C);
            int rc = mpfft_shard_stage(MPFFT_SHARD_FWD_COLUMNS, &sh, R.src[0] + e * sl, R.src[1] + e * sl, R.s);
            if (rc) return rc;
            for (const mpfft_copy &c : plan)
                if (c.dst == d && c.src == e) {
                    mpfft_copy m = c;
                    m.src = d;          // block e's column layout is rank d's own column arrays now
                    if ((rc = queue_copy(rk, m, R.s))) return rc;
                }
        }
        MCHK(hipEventRecord(R.ev, R.s));
    }
    return MPFFT_OK;
}

int run_exchange_fwd(const Part &p, std::vector<Rank> &rk)
{
    std::vector<mpfft_copy> plan;
    exchange_plan(p, MPFFT_XCHG_COL_TO_ROW, plan);
    for (int d = 0; d < p.world; ++d) {
        Rank &D = rk[d];
        MCHK(hipSetDevice(D.dev));
        for (int op = 0; op < 2; ++op) {
            for (int s = 0; s < p.world; ++s) MCHK(hipStreamWaitEvent(D.xs, op ? rk[s].ev : rk[s].eva, 0));
            for (const mpfft_copy &c : plan)
                if (c.dst == d && c.op == op) {
                    int rc = queue_copy(rk, c, D.xs);
                    if (rc) return rc;
                }
        }
        MCHK(hipEventRecord(D.evx, D.xs));
    }
    for (int d = 0; d < p.world; ++d) {   // senders' compute streams must not run ahead of the pulls
        MCHK(hipSetDevice(rk[d].dev));
        for (int s = 0; s < p.world; ++s) MCHK(hipStreamWaitEvent(rk[d].s, rk[s].evx, 0));
        MCHK(hipEventRecord(rk[d].ev, rk[d].s));
    }
    return MPFFT_OK;
}

// queue one exchange: each receiver waits for every sender's last event, then pulls
int run_exchange(const Part &p, std::vector<Rank> &rk, int which)
{
    std::vector<mpfft_copy> plan;
    exchange_plan(p, which, plan);
    for (int d = 0; d < p.world; ++d) {
        MCHK(hipSetDevice(rk[d].dev));
        for (int s = 0; s < p.world; ++s)
            if (s != d) MCHK(hipStreamWaitEvent(rk[d].s, rk[s].ev, 0));
        for (const mpfft_copy &c : plan) {
            if (c.dst != d) continue;
            int rc = queue_copy(rk, c, rk[d].s);
            if (rc) return rc;
        }
    }
    for (int d = 0; d < p.world; ++d) {
        MCHK(hipSetDevice(rk[d].dev));
        MCHK(hipEventRecord(rk[d].ev, rk[d].s));
    }
    return MPFFT_OK;
}

int stage_all(const Part &p, std::vector<Rank> &rk, int stage, unsigned long depth, unsigned long w,
              bool ev_a = false)
{
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        MCHK(hipSetDevice(R.dev));
        const mpfft_shard sh = desc(p, d, R, depth, w);
        int rc = mpfft_shard_stage(stage, &sh, R.src[0], R.src[1], R.s);
        if (rc) return rc;
        if (stage == MPFFT_SHARD_POINTWISE && p.fused) {   // the product is in rowc: operand 0 from here on
            std::swap(R.row[0], R.rowc);
            if (p.world == 1) std::swap(R.col[0], R.colc);
        }
        MCHK(hipEventRecord(ev_a ? R.eva : R.ev, R.s));
    }
    return MPFFT_OK;
}

void enable_peers(const std::vector<int> &devs)
{
    for (int a : devs)
        for (int b : devs) {
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can && hipSetDevice(a) == hipSuccess) {
                const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess) (void)hipGetLastError();   // already enabled: fine
            }
        }
}

int mul_multi_locked(Ctx &X, uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2,
                     unsigned long depth, unsigned long w, const std::vector<int> &devs)
{
    Part p;
    const int G = (int)devs.size();
    int rc = partition(p, n1, n2, depth, w, G);
    if (rc) return rc;
    // replicated forward columns at two ranks (sharded.py ShardedMul.replicates: exchange #1
    // there is one xGMI link carrying the other rank's rows of both column blocks; the second column block
    // is one more column phase of HBM-bound passes); MPFFT_REPLICATE_COLUMNS=0/1 overrides
    {
        const char *e = getenv("MPFFT_REPLICATE_COLUMNS");
        p.rep = e ? (e[0] == '1' && G > 1) : G == 2;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return MPFFT_ENODEV;
    for (int d : devs)
        if (d < 0 || d >= ndev) return MPFFT_ENODEV;
    if (X.devs != devs) {
        for (Rank &R : X.ranks) free_rank(R);
        X.ranks.assign(G, Rank());
        for (int g = 0; g < G; ++g) X.ranks[g].dev = devs[g];
        X.devs = devs;
        enable_peers(devs);
    }
    std::vector<Rank> &rk = X.ranks;
    for (int d = 0; d < G; ++d)
        if ((rc = setup_rank(p, d, rk[d]))) return rc;

    // operand slices: packed and copied by one host thread per rank
    std::vector<int> trc(G, MPFFT_OK);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < G; ++d)
            th.emplace_back([&, d] {
                Rank &R = rk[d];
                const long sl = p.Tr * p.chunk, ns = p.nsl();
                u64 *h0 = R.host, *h1 = R.host + ns * sl;
                for (long e = 0; e < ns; ++e) {   // replicated: every block's slices, block e at e sl
                    const int blk = p.rep ? (int)e : d;
                    pack_slice(p, blk, i1, n1, h0 + e * sl);
                    pack_slice(p, blk, i2, n2, h1 + e * sl);
                }
                if (hipSetDevice(R.dev) != hipSuccess ||
                    hipMemcpyAsync(R.src[0], h0, (size_t)ns * sl * 8, hipMemcpyHostToDevice, R.s) != hipSuccess ||
                    hipMemcpyAsync(R.src[1], h1, (size_t)ns * sl * 8, hipMemcpyHostToDevice, R.s) != hipSuccess)
                    trc[d] = MPFFT_EHIP;
            });
        for (auto &t : th) t.join();
        for (int d = 0; d < G; ++d)
            if (trc[d]) return trc[d];
    }

    if (p.rep) {
        if ((rc = fwd_replicated(p, rk, depth, w))) return rc;
    } else {
        if ((rc = stage_all(p, rk, MPFFT_SHARD_FWD_COLUMNS_A, depth, w, true))) return rc;
        if ((rc = stage_all(p, rk, MPFFT_SHARD_FWD_COLUMNS_B, depth, w))) return rc;
        if ((rc = run_exchange_fwd(p, rk))) return rc;
    }
    if ((rc = stage_all(p, rk, MPFFT_SHARD_FWD_ROWS, depth, w))) return rc;
    if ((rc = stage_all(p, rk, MPFFT_SHARD_POINTWISE, depth, w))) return rc;
    if ((rc = stage_all(p, rk, MPFFT_SHARD_INV_ROWS, depth, w))) return rc;
    if ((rc = run_exchange(p, rk, MPFFT_XCHG_ROW_TO_COL))) return rc;
    if ((rc = stage_all(p, rk, MPFFT_SHARD_INV_COLUMNS, depth, w))) return rc;
    if ((rc = run_exchange(p, rk, MPFFT_XCHG_COEFFS))) return rc;

    // halo: the last H coefficients of rank d-1's range (its row layout) -> rank d
    for (int d = 1; d < G; ++d) {
        Rank &R = rk[d], &S = rk[d - 1];
        MCHK(hipSetDevice(R.dev));
        MCHK(hipStreamWaitEvent(R.s, S.ev, 0));
        const long r0 = p.rows[d - 1], rc_ = p.rcount(d - 1), kend = p.rows[d] * p.NC;
        for (long h = 0; h < p.H; ++h) {
            const long k = kend - p.H + h, pp = k / p.NC - r0, cc = k % p.NC;
            const long slot = (cc / p.C) * (rc_ * p.C) + pp * p.C + (cc % p.C);
            const u64 *sp = S.row[0].dig + slot * p.l;
            u64 *dp = R.halo + h * p.l;
            if (S.dev == R.dev) MCHK(hipMemcpyAsync(dp, sp, (size_t)p.l * 8, hipMemcpyDeviceToDevice, R.s));
            else MCHK(hipMemcpyPeerAsync(dp, R.dev, sp, S.dev, (size_t)p.l * 8, R.s));
        }
    }

    // combine phase 0, the cross-rank carry (generate, propagate per rank), phase 1
    std::vector<int> sums(2 * G, 0);
    for (int d = 0; d < G; ++d) {
        Rank &R = rk[d];
        MCHK(hipSetDevice(R.dev));
        const mpfft_shard sh = desc(p, d, R, depth, w);
        const long mcount = p.M[d + 1] - p.M[d];
        if (mcount < 1) continue;
        rc = mpfft_shard_combine(&sh, 0, R.r, p.M[d], mcount, p.rows[d] * p.NC, d ? R.halo : nullptr,
                                 d ? (int)p.H : 0, R.tmp, R.tmp_bytes, 0, R.sum, R.s);
        if (rc) return rc;
        MCHK(hipMemcpyAsync(&sums[2 * d], R.sum, 2 * sizeof(int), hipMemcpyDeviceToHost, R.s));
    }
    for (int d = 0; d < G; ++d) {
        MCHK(hipSetDevice(rk[d].dev));
        MCHK(hipStreamSynchronize(rk[d].s));
    }
    int cin = 0;
    for (int d = 0; d < G; ++d) {
        Rank &R = rk[d];
        const long mcount = p.M[d + 1] - p.M[d];
        if (mcount >= 1 && cin) {
            MCHK(hipSetDevice(R.dev));
            const mpfft_shard sh = desc(p, d, R, depth, w);
            rc = mpfft_shard_combine(&sh, 1, R.r, p.M[d], mcount, p.rows[d] * p.NC, d ? R.halo : nullptr,
                                     d ? (int)p.H : 0, R.tmp, R.tmp_bytes, 1, R.sum, R.s);
            if (rc) return rc;
        }
        if (mcount >= 1) cin = (sums[2 * d] || (sums[2 * d + 1] && cin)) ? 1 : 0;
    }
    // product limbs: one thread per rank (pageable destination)
    {
        std::vector<std::thread> th;
        for (int d = 0; d < G; ++d)
            th.emplace_back([&, d] {
                Rank &R = rk[d];
                const long mcount = p.M[d + 1] - p.M[d];
                if (hipSetDevice(R.dev) != hipSuccess) { trc[d] = MPFFT_EHIP; return; }
                if (mcount > 0 && hipMemcpyAsync(r1 + p.M[d], R.r, (size_t)mcount * 8, hipMemcpyDeviceToHost, R.s) != hipSuccess)
                    trc[d] = MPFFT_EHIP;
                if (hipStreamSynchronize(R.s) != hipSuccess) trc[d] = MPFFT_EHIP;
            });
        for (auto &t : th) t.join();
        for (int d = 0; d < G; ++d)
            if (trc[d]) return trc[d];
    }
    return MPFFT_OK;
}

struct Policy {
    std::mutex mu;
    bool init = false;
    std::vector<int> devs;
    long min_l = 1024;
};
Policy g_pol;

void policy_init_locked()
{
    if (g_pol.init) return;
    g_pol.init = true;
    const char *e = getenv("MPFFT_DEVICES");
    if (!e || !*e) return;
    std::vector<int> v;
    const char *q = e;
    while (*q) {
        char *end = nullptr;
        const long d = strtol(q, &end, 10);
        if (end == q) break;
        v.push_back((int)d);
        q = *end == ',' ? end + 1 : end;
        if (*end != ',') break;
    }
    if (v.size() > 1) g_pol.devs = v;
}

}  // namespace

// used by mpfft_mul_ex (mpfft.hip): the device list the policy picks for this product, if any
int mpfft_multi_policy(long n1, long n2, unsigned long depth, unsigned long w, std::vector<int> &devs)
{
    {
        std::lock_guard<std::mutex> lk(g_pol.mu);
        policy_init_locked();
        if (g_pol.devs.size() < 2) return 0;
        devs = g_pol.devs;
    }
    long info[10];
    if (mpfft_plan_info(n1, n2, depth, w, info) || info[1] < g_pol.min_l) return 0;
    Part p;
    return partition(p, n1, n2, depth, w, (int)devs.size()) == MPFFT_OK ? (int)devs.size() : 0;
}

extern "C" {

int mpfft_shard_partition(long n1, long n2, unsigned long depth, unsigned long w, int world, long *rows, long *M,
                          long *info)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return rc;
    for (int d = 0; d <= world; ++d) {
        rows[d] = p.rows[d];
        M[d] = p.M[d];
    }
    info[0] = p.C;
    info[1] = p.chunk;
    info[2] = p.H;
    info[3] = p.Tr;
    info[4] = p.fused ? 1 : 0;
    return MPFFT_OK;
}

long mpfft_shard_exchange_plan(long n1, long n2, unsigned long depth, unsigned long w, int world, int which,
                               mpfft_copy *out, long cap)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return -rc;
    if (which < MPFFT_XCHG_COL_TO_ROW || which > MPFFT_XCHG_COEFFS) return -MPFFT_EINVAL;
    std::vector<mpfft_copy> v;
    exchange_plan(p, which, v);
    if (out) {
        if (cap < (long)v.size()) return -MPFFT_EINVAL;
        memcpy(out, v.data(), v.size() * sizeof(mpfft_copy));
    }
    return (long)v.size();
}

int mpfft_mul_multi(uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2, unsigned long depth,
                    unsigned long w, int ngpus, const int *devices)
{
    if (ngpus < 1) return MPFFT_EINVAL;
    std::vector<int> devs(ngpus);
    for (int g = 0; g < ngpus; ++g) devs[g] = devices ? devices[g] : g;
    int cur = 0;
    (void)hipGetDevice(&cur);
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    (void)hipGetLastError();
    const int rc = mul_multi_locked(g_ctx, r1, i1, n1, i2, n2, depth, w, devs);
    if (rc) {   // leave no work queued behind a failed call
        for (Rank &R : g_ctx.ranks)
            if (R.s) {
                (void)hipSetDevice(R.dev);
                (void)hipStreamSynchronize(R.s);
            }
    }
    (void)hipSetDevice(cur);
    return rc;
}

int mpfft_multi_release(void)
{
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (Rank &R : g_ctx.ranks) free_rank(R);
    g_ctx.ranks.clear();
    g_ctx.devs.clear();
    (void)hipSetDevice(cur);
    return MPFFT_OK;
}

int mpfft_set_devices(int ngpus, const int *devices, long min_l)
{
    std::lock_guard<std::mutex> lk(g_pol.mu);
    g_pol.init = true;   // an explicit choice overrides MPFFT_DEVICES
    g_pol.devs.clear();
    if (ngpus > 1) {
        for (int g = 0; g < ngpus; ++g) g_pol.devs.push_back(devices ? devices[g] : g);
    }
    g_pol.min_l = min_l > 0 ? min_l : 1024;
    return MPFFT_OK;
}

}  // extern "C"
