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
//   halo      the H coefficients before each of the rank's stripes (a few per row position)
//   combine   in the column layout: rank g's C columns of row position j are product stripe
//             j G + g (C consecutive coefficients, a contiguous bit range), combined with
//             carry-in 0 (phase 0); every rank's stripe summaries to every rank (peer copies of
//             Tr (generate, propagate) pairs); phase 1 adds each stripe's carry-in on the device
//   D2H       rank g's stripes into their places in r1 (one thread per rank)
//
// The product never moves back to row owners: the combine needs only each stripe's few halo
// coefficients (the reference's TODO:53-59, "combine just a single coefficient at a time so
// that cache locality can be maintained for the MFA IFFT's").
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

#include <stdarg.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpfft.h"

typedef uint64_t u64;

void mpfft_note_hip_error(hipError_t e);   // mpfft.c: what mpfft_strerror(MPFFT_EHIP) reports

namespace {

struct Part {
    int world;
    unsigned long depth, w;
    long n1, n2, total, n, l, NC, NR, T, Tr, bits1, N, len;
    long C, chunk, H, cbw;
    long S, SL;    // product stripes (world Tr) and the most limbs of one (the combine's d_r stride)
    bool fused;
    bool rep;      // replicated forward columns: every rank computes every column block (world 2)
    long nsl() const { return rep ? world : 1; }   // operand column slices a rank holds
    long src_limbs() const { return nsl() * Tr * chunk; }
    std::vector<long> rows, ms;   // ms[s]: first product limb of stripe s (combine.hpp stripe_m)
    long rcount(int d) const { return rows[d + 1] - rows[d]; }
};

long cb_words_l(long l) { return 2 * ((l + 63) / 64); }

// replicated forward columns at two ranks (sharded.py ShardedMul.replicates: exchange #1 there
// is one xGMI link carrying the other rank's rows of both column blocks; the second column
// block is one more column phase of HBM-bound passes); MPFFT_REPLICATE_COLUMNS=0/1 overrides
bool replicated(int world)
{
    const char *e = getenv("MPFFT_REPLICATE_COLUMNS");
    return e ? (e[0] == '1' && world > 1) : world == 2;
}

// ShardPlan (sharded.py) in C: the same arithmetic, so both drivers agree slot for slot
int partition(Part &p, long n1, long n2, unsigned long depth, unsigned long w, int world)
{
    long info[10];
    int rc = mpfft_plan_info(n1, n2, depth, w, info);
    if (rc) return rc;
    p.world = world;
    p.depth = depth;
    p.w = w;
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
    if (p.Tr < world) return MPFFT_EINVAL;
    for (int d = 0; d < world; ++d)
        if (p.rows[d + 1] - p.rows[d] < 1) return MPFFT_EINVAL;  // a rank without rows
    p.H = (p.N + 128 + p.bits1 - 1) / p.bits1 + 1;
    p.cbw = cb_words_l(p.l);
    p.chunk = (p.C * p.bits1 + 63) / 64 + 2;
    p.fused = mpfft_shard_row_fused(n1, n2, depth, w, (int)p.C) != 0;
    p.rep = replicated(world);
    p.S = (long)world * p.Tr;
    p.SL = (long)((((u64)p.C + 1) * (u64)p.bits1) / 64) + 2;   // mpfft.hip shard_comb_args
    p.ms.assign(p.S + 1, p.total);
    for (long s = 0; s < p.S; ++s) {
        const long m = (long)(((u64)s * (u64)p.C * (u64)p.bits1) >> 6);
        p.ms[s] = m < p.total ? m : p.total;
    }
    return MPFFT_OK;
}

long field_width(const Part &p, int f) { return f == 0 ? p.l : f == 1 ? p.cbw : 1; }

// the copies of one exchange (sharded.py ShardedMul._exchange): #1 column layout rows
// [rows[d], rows[d+1]) -> rank d's row layout (both operands), #2 the product back
void exchange_plan(const Part &p, int which, std::vector<mpfft_copy> &out)
{
    out.clear();
    const int nf = 3;
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

// the halo copies (sharded.py ShardedMul._halo): for stripe s = j G + g, coefficients
// [s C - H, s C) from the ranks holding them (stripe t = k / C: rank t % G, column-layout
// slot (t / G) C + k % C) to rank g's halo slot j H + k - (s C - H), split into runs of one
// source stripe; offsets and counts in limbs
void halo_plan(const Part &p, std::vector<mpfft_copy> &out)
{
    out.clear();
    for (int g = 0; g < p.world; ++g)
        for (long j = 0; j < p.Tr; ++j) {
            const long s = j * p.world + g, k1 = s * p.C, k0 = k1 - p.H;
            for (long k = k0 > 0 ? k0 : 0; k < k1;) {
                const long t = k / p.C, ke = (t + 1) * p.C < k1 ? (t + 1) * p.C : k1;
                const long src_slot = (t / p.world) * p.C + k % p.C, dst_slot = j * p.H + (k - k0);
                mpfft_copy c = {(int)(t % p.world), g, 0, 0, 0, MPFFT_LAYOUT_HALO, src_slot * p.l, dst_slot * p.l,
                                (ke - k) * p.l};
                out.push_back(c);
                k = ke;
            }
        }
}

// A run of limbs copied by k_copy_runs: src offset -> dst offset, n limbs
struct Run {
    long src, dst, n;
};

// one workgroup per run (grid-stride): the halo's pack on the sender (column layout -> one
// contiguous block per receiver) and, where a receiver's runs from one sender are not
// contiguous in its halo, the scatter from its staging buffer
__global__ __launch_bounds__(256) void k_copy_runs(const Run *runs, long nruns, const u64 *src, u64 *dst)
{
    for (long r = blockIdx.x; r < nruns; r += gridDim.x) {
        const Run R = runs[r];
        for (long i = threadIdx.x; i < R.n; i += blockDim.x) dst[R.dst + i] = src[R.src + i];
    }
}

// the halo plan as transfers: per sender one pack launch into its send block (grouped by
// receiver), one peer copy per (sender, receiver) pair -- straight into the receiver's halo
// when that sender's runs are contiguous there (always when H <= C: stripe j G + g's halo is
// the tail of stripe j G + g - 1), else into a staging block the receiver scatters
struct HaloRank {
    std::vector<Run> pack, scatter;
    long send_n = 0, stage_n = 0;
    std::vector<long> send_off, send_cnt;   // per receiver: its block of the send buffer
    std::vector<long> recv_halo;            // per sender: halo offset of its block, or -1: staging
    std::vector<long> recv_stage;           // per sender: staging offset of its block
};

void halo_xfer(const Part &p, std::vector<HaloRank> &hr)
{
    std::vector<mpfft_copy> plan;
    halo_plan(p, plan);
    const int G = p.world;
    hr.assign(G, HaloRank());
    for (int s = 0; s < G; ++s) {
        HaloRank &S = hr[s];
        S.send_off.assign(G, 0);
        S.send_cnt.assign(G, 0);
        for (int d = 0; d < G; ++d) {
            S.send_off[d] = S.send_n;
            for (const mpfft_copy &c : plan)
                if (c.src == s && c.dst == d) {
                    S.pack.push_back({c.src_off, S.send_n, c.count});
                    S.send_n += c.count;
                }
            S.send_cnt[d] = S.send_n - S.send_off[d];
        }
    }
    for (int d = 0; d < G; ++d) {
        HaloRank &D = hr[d];
        D.recv_halo.assign(G, -1);
        D.recv_stage.assign(G, 0);
        for (int s = 0; s < G; ++s) {
            long first = -1, next = -1, n = 0;
            bool contiguous = true;
            for (const mpfft_copy &c : plan)
                if (c.src == s && c.dst == d) {
                    if (first < 0) first = c.dst_off;
                    else if (c.dst_off != next) contiguous = false;
                    next = c.dst_off + c.count;
                    n += c.count;
                }
            if (!n) continue;
            if (contiguous) {
                D.recv_halo[s] = first;
                continue;
            }
            D.recv_stage[s] = D.stage_n;
            long o = D.stage_n;
            for (const mpfft_copy &c : plan)
                if (c.src == s && c.dst == d) {
                    D.scatter.push_back({o, c.dst_off, c.count});
                    o += c.count;
                }
            D.stage_n = o;
        }
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
    hipEvent_t evs = nullptr;    // combine phase 0 done: this rank's stripe summaries are ready
    hipEvent_t evd = nullptr;    // this rank's whole call done (every pull it made is complete)
    bool done_rec = false;       // evd recorded by an earlier call
    unsigned char *mem = nullptr;
    size_t mem_bytes = 0;
    u64 *host = nullptr;      // pinned staging of the operand slices
    size_t host_bytes = 0;
    Arr col[2], row[2], colc, rowc;
    u64 *src[2] = {nullptr, nullptr};   // the host entry's operand slices (H2D)
    u64 *halo = nullptr, *r = nullptr;  // the stripes' halo coefficients; the host entry's product stripes
    int *sums = nullptr, *sums_all = nullptr;   // this rank's stripe summaries; every rank's
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    const u64 *in[2] = {nullptr, nullptr};   // this call's operand slices
    bool whole = false;                      // ... or the whole operands (host entry, replicated columns)
    u64 *out = nullptr;                      // this call's product stripes
    u64 *hsend = nullptr, *hstage = nullptr;  // the halo's send block and staging (HaloRank)
    Run *d_pack = nullptr, *d_scatter = nullptr;   // its run tables on the device
    std::vector<long> tables_key;            // the partition whose tables are uploaded
};

struct Ctx {
    std::mutex mu;
    std::vector<int> devs;
    std::vector<Rank> ranks;
    std::vector<long> key;           // the partition the halo transfers below belong to
    std::vector<HaloRank> halo;
};

std::vector<long> part_key(const Part &p)
{
    return {p.n1, p.n2, (long)p.depth, (long)p.w, p.world, p.rep ? 1 : 0};
}
Ctx g_ctx;

#define MCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { mpfft_note_hip_error(e_); return MPFFT_EHIP; } } while (0)

// ---- the event graph ------------------------------------------------------------------------
// Every cross-stream ordering in run_ranks goes through rec() / wait() and every queued piece of
// work through work() / copy_from(): with a schedule trace active they also append one line to
// it, and in a dry run (mpfft_multi_schedule) they do only that -- no HIP call, no memory -- so
// the CPU tests check the event graph itself (tests/test_multi_schedule.py):
//   R d S E       record rank d's event E on its stream S (s: compute, x: exchange #1)
//   W d S e E     rank d's stream S waits for rank e's event E (its most recent record)
//   K d S what    work on rank d's stream S that touches rank d's buffers only
//   C d S what e  a copy on rank d's stream S reading rank e's buffers into rank d's
//   N             the next call
enum { EV_MAIN, EV_A, EV_X, EV_SUM, EV_DONE };
const char *const ev_names[] = {"ev", "eva", "evx", "evs", "evd"};
struct Sched {
    std::string log;
    bool dry = false;
};
thread_local Sched *g_sched = nullptr;
bool dry() { return g_sched && g_sched->dry; }
void sched_line(const char *fmt, ...)
{
    if (!g_sched) return;
    char b[160];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof(b), fmt, ap);
    va_end(ap);
    g_sched->log += b;
    g_sched->log += '\n';
}
hipEvent_t ev_of(const Rank &R, int e)
{
    return e == EV_MAIN ? R.ev : e == EV_A ? R.eva : e == EV_X ? R.evx : e == EV_SUM ? R.evs : R.evd;
}
#define SETDEV(R) do { if (!dry()) MCHK(hipSetDevice((R).dev)); } while (0)
int rec(std::vector<Rank> &rk, int d, int e, bool xs = false)
{
    sched_line("R %d %c %s", d, xs ? 'x' : 's', ev_names[e]);
    if (!dry()) MCHK(hipEventRecord(ev_of(rk[d], e), xs ? rk[d].xs : rk[d].s));
    return MPFFT_OK;
}
int wait(std::vector<Rank> &rk, int d, bool xs, int e, int ev)
{
    sched_line("W %d %c %d %s", d, xs ? 'x' : 's', e, ev_names[ev]);
    if (!dry()) MCHK(hipStreamWaitEvent(xs ? rk[d].xs : rk[d].s, ev_of(rk[e], ev), 0));
    return MPFFT_OK;
}
bool work(int d, bool xs, const char *what)   // false: a dry run (skip the HIP call)
{
    sched_line("K %d %c %s", d, xs ? 'x' : 's', what);
    return !dry();
}
bool copy_from(int d, bool xs, const char *what, int src)
{
    sched_line("C %d %c %s %d", d, xs ? 'x' : 's', what, src);
    return !dry();
}

size_t al(size_t x) { return (x + 255) / 256 * 256; }

// wait for every stream of every rank: no copy engine may still read or write a buffer
// that is about to be freed (another rank's exchange stream may be pulling from it)
void drain(std::vector<Rank> &rk)
{
    for (Rank &R : rk) {
        if (!R.s && !R.xs) continue;
        (void)hipSetDevice(R.dev);
        if (R.s) (void)hipStreamSynchronize(R.s);
        if (R.xs) (void)hipStreamSynchronize(R.xs);
    }
}

// after drain(rk)
void free_rank(Rank &R)
{
    if (R.s || R.mem || R.host) (void)hipSetDevice(R.dev);
    if (R.mem) (void)hipFree(R.mem);
    if (R.host) (void)hipHostFree(R.host);
    if (R.ev) (void)hipEventDestroy(R.ev);
    if (R.eva) (void)hipEventDestroy(R.eva);
    if (R.evx) (void)hipEventDestroy(R.evx);
    if (R.evs) (void)hipEventDestroy(R.evs);
    if (R.evd) (void)hipEventDestroy(R.evd);
    if (R.s) (void)hipStreamDestroy(R.s);
    if (R.xs) (void)hipStreamDestroy(R.xs);
    R = Rank();
}

// rank d's device bytes (one grow-only allocation) and pinned host bytes for partition p
size_t rank_need(const Part &p, int d, bool host, const HaloRank &HR, size_t *host_bytes)
{
    const long cs = p.NR * p.C, rs = p.rcount(d) * p.NC;
    const bool w1 = p.world == 1;
    const int ncol = (w1 && p.fused) ? 3 : 2;          // world 1: the fused product's column array
    const int nrow = w1 ? 0 : (p.fused ? 3 : 2);      // world 1: row arrays are views
    auto arr_bytes = [&](long slots) { return al(slots * p.l * 8) + al(slots * p.cbw * 8) + al(slots * 4); };
    const size_t ctb = mpfft_shard_combine_tmp_bytes(p.n1, p.n2, p.depth, p.w, p.world);
    // the host entry's device copies of its operands: the rank's slices, or the whole operands
    // when every rank computes every column block (no packing: straight H2D)
    const long s1 = p.rep ? p.n1 : p.src_limbs(), s2 = p.rep ? p.n2 : p.src_limbs();
    *host_bytes = host ? (size_t)std::max<long>(p.rep ? 0 : 2 * p.src_limbs(), p.Tr * p.SL) * 8 : 0;
    return ncol * arr_bytes(cs) + nrow * arr_bytes(rs) + (host ? al(s1 * 8) + al(s2 * 8) + al(p.Tr * p.SL * 8) : 0) +
           al(p.Tr * p.H * p.l * 8) + al(p.Tr * 2 * 4) + al(p.world * p.Tr * 2 * 4) + al(ctb) +
           al(HR.send_n * 8) + al(HR.stage_n * 8) + al(HR.pack.size() * sizeof(Run)) +
           al(HR.scatter.size() * sizeof(Run)) + 256;
}

// carve rank d's arrays out of one grow-only allocation (host: also the operand slices, their
// pinned staging and the product stripes).  A reallocation frees memory other ranks' streams
// may still pull from: prepare() drains every rank first when any of them grows.
int setup_rank(const Part &p, int d, Rank &R, bool host, const HaloRank &HR)
{
    MCHK(hipSetDevice(R.dev));
    if (!R.s) MCHK(hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking));
    if (!R.ev) MCHK(hipEventCreateWithFlags(&R.ev, hipEventDisableTiming));
    if (!R.xs) MCHK(hipStreamCreateWithFlags(&R.xs, hipStreamNonBlocking));
    if (!R.eva) MCHK(hipEventCreateWithFlags(&R.eva, hipEventDisableTiming));
    if (!R.evx) MCHK(hipEventCreateWithFlags(&R.evx, hipEventDisableTiming));
    if (!R.evs) MCHK(hipEventCreateWithFlags(&R.evs, hipEventDisableTiming));
    if (!R.evd) MCHK(hipEventCreateWithFlags(&R.evd, hipEventDisableTiming));
    const long cs = p.NR * p.C, rs = p.rcount(d) * p.NC;
    const bool w1 = p.world == 1;
    const int ncol = (w1 && p.fused) ? 3 : 2;
    const long s1 = p.rep ? p.n1 : p.src_limbs(), s2 = p.rep ? p.n2 : p.src_limbs();
    size_t hb = 0;
    const size_t need = rank_need(p, d, host, HR, &hb);
    const size_t ctb = mpfft_shard_combine_tmp_bytes(p.n1, p.n2, p.depth, p.w, p.world);
    if (R.mem_bytes < need) {
        if (R.mem) {
            (void)hipStreamSynchronize(R.s);
            MCHK(hipFree(R.mem));
        }
        R.mem = nullptr;
        R.mem_bytes = 0;
        if (hipMalloc((void **)&R.mem, need) != hipSuccess) {
            (void)hipGetLastError();
            return MPFFT_ENOMEM;
        }
        R.mem_bytes = need;
        R.tables_key.clear();
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
    R.halo = (u64 *)q; q += al(p.Tr * p.H * p.l * 8);
    R.sums = (int *)q; q += al(p.Tr * 2 * 4);
    R.sums_all = (int *)q; q += al(p.world * p.Tr * 2 * 4);
    R.tmp = q; q += al(ctb);
    R.tmp_bytes = ctb;
    R.hsend = (u64 *)q; q += al(HR.send_n * 8);
    R.hstage = (u64 *)q; q += al(HR.stage_n * 8);
    R.d_pack = (Run *)q; q += al(HR.pack.size() * sizeof(Run));
    R.d_scatter = (Run *)q; q += al(HR.scatter.size() * sizeof(Run));
    const std::vector<long> key = part_key(p);
    if (R.tables_key != key) {   // the run tables: once per partition (the carve is deterministic)
        if (!HR.pack.empty())
            MCHK(hipMemcpyAsync(R.d_pack, HR.pack.data(), HR.pack.size() * sizeof(Run), hipMemcpyHostToDevice, R.s));
        if (!HR.scatter.empty())
            MCHK(hipMemcpyAsync(R.d_scatter, HR.scatter.data(), HR.scatter.size() * sizeof(Run),
                                hipMemcpyHostToDevice, R.s));
        MCHK(hipStreamSynchronize(R.s));   // (pageable sources)
        R.tables_key = key;
    }
    if (host) {
        R.src[0] = (u64 *)q; q += al(s1 * 8);
        R.src[1] = (u64 *)q; q += al(s2 * 8);
        R.r = (u64 *)q; q += al(p.Tr * p.SL * 8);
        // pinned staging: the packed slices on the way in, the stripes on the way out (hb)
        if (R.host_bytes < hb) {
            if (R.host) MCHK(hipHostFree(R.host));
            R.host = nullptr;
            R.host_bytes = 0;
            if (hipHostMalloc((void **)&R.host, hb, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                return MPFFT_ENOMEM;
            }
            R.host_bytes = hb;
        }
    } else {
        R.src[0] = R.src[1] = nullptr;
        R.r = nullptr;
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
    sh.src_chunk = R.whole ? 0 : p.chunk;
    if (p.fused) {
        sh.rowc_dig = R.rowc.dig;
        sh.rowc_cb = R.rowc.cb;
        sh.rowc_top = R.rowc.top;
    }
    return sh;
}

// rank d's column slices of operand a: for each live row position q, `chunk` limbs from limb
// floor((q NC + blk C) bits1 / 64) on (ShardPlan.slice_operand), for its own column block, or
// for every block in turn when the forward columns are replicated
void pack_slices(const Part &p, int d, const u64 *a, long na, u64 *out)
{
    for (long e = 0; e < p.nsl(); ++e) {
        const long blk = p.rep ? e : d;
        for (long q = 0; q < p.Tr; ++q) {
            u64 *o = out + (e * p.Tr + q) * p.chunk;
            const long s0 = (long)(((unsigned __int128)(q * p.NC + blk * p.C) * (u64)p.bits1) / 64);
            long cnt = 0;
            if (s0 < na) {
                cnt = na - s0 < p.chunk ? na - s0 : p.chunk;
                memcpy(o, a + s0, (size_t)cnt * 8);
            }
            if (cnt < p.chunk) memset(o + cnt, 0, (size_t)(p.chunk - cnt) * 8);
        }
    }
}

void *field_ptr(const Arr &a, int f, long off)
{
    if (f == 0) return a.dig + off;
    if (f == 1) return a.cb + off;
    return a.top + off;
}

void *loc(const Rank &R, int layout, int op, int field, long off)
{
    if (layout == MPFFT_LAYOUT_HALO) return R.halo + off;
    return field_ptr(layout ? R.row[op] : R.col[op], field, off);
}

// queue one copy of an exchange or halo plan on its receiving rank's stream (xs: the exchange
// stream)
int queue_copy(std::vector<Rank> &rk, const mpfft_copy &c, bool xs, const char *what)
{
    const Rank &S = rk[c.src], &D = rk[c.dst];
    const size_t es = c.field == 2 ? 4 : 8;
    if (dry()) {   // a dry run has no buffers
        copy_from(c.dst, xs, what, c.src);
        return MPFFT_OK;
    }
    void *dp = loc(D, c.dst_layout, c.op, c.field, c.dst_off);
    const void *sp = loc(S, c.src_layout, c.op, c.field, c.src_off);
    if (dp == sp) return MPFFT_OK;   // world 1: the row layout is a view of the column layout
    copy_from(c.dst, xs, what, c.src);
    const hipStream_t st = xs ? D.xs : D.s;
    if (S.dev == D.dev) MCHK(hipMemcpyAsync(dp, sp, c.count * es, hipMemcpyDeviceToDevice, st));
    else MCHK(hipMemcpyPeerAsync(dp, D.dev, sp, S.dev, c.count * es, st));
    return MPFFT_OK;
}

const char *shard_stage_name(int stage)
{
    switch (stage) {
    case MPFFT_SHARD_FWD_COLUMNS_A: return "fwd_columns_a";
    case MPFFT_SHARD_FWD_COLUMNS_B: return "fwd_columns_b";
    case MPFFT_SHARD_FWD_COLUMNS_OWN: return "fwd_columns_own";
    case MPFFT_SHARD_FWD_ROWS: return "fwd_rows";
    case MPFFT_SHARD_POINTWISE: return "pointwise";
    case MPFFT_SHARD_INV_ROWS: return "inv_rows";
    case MPFFT_SHARD_INV_COLUMNS: return "inv_columns";
    }
    return "stage";
}

// replicated forward columns (world 2): rank d runs every column block e's split + column
// passes from block e's operand slices into its own column arrays (scratch) -- for its own
// rows only: after the first pass the passes skip the DIF subtrees that hold none of them
// (MPFFT_SHARD_FWD_COLUMNS_OWN) -- then plays exchange #1's copies from e to d locally: its
// rows of block e into its row layout
int fwd_replicated(const Part &p, std::vector<Rank> &rk, unsigned long depth, unsigned long w)
{
    std::vector<mpfft_copy> plan;
    exchange_plan(p, MPFFT_XCHG_COL_TO_ROW, plan);
    const long sl = p.Tr * p.chunk;
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        SETDEV(R);
        for (int e = 0; e < p.world; ++e) {
            mpfft_shard sh = desc(p, d, R, depth, w);
            sh.c0 = (int)(e * p.C);
            const long o = R.whole ? 0 : e * sl;   // block e's slices, or the whole operands
            int rc;
            if (work(d, false, shard_stage_name(MPFFT_SHARD_FWD_COLUMNS_OWN)) &&
                (rc = mpfft_shard_stage(MPFFT_SHARD_FWD_COLUMNS_OWN, &sh, R.in[0] + o, R.in[1] + o, R.s)))
                return rc;
            for (const mpfft_copy &c : plan)
                if (c.dst == d && c.src == e) {
                    mpfft_copy m = c;
                    m.src = d;          // block e's column layout is rank d's own column arrays now
                    if ((rc = queue_copy(rk, m, false, "xchg1_local"))) return rc;
                }
        }
        if (int rc = rec(rk, d, EV_MAIN)) return rc;
    }
    return MPFFT_OK;
}

// exchange #1 with the forward column passes run per operand: every receiver's exchange
// stream pulls operand 1's blocks once all senders finished operand 1's passes (event eva)
// -- while the compute streams run operand 2's passes -- then operand 2's (event ev); the
// compute stream waits for both before the row passes
int run_exchange_fwd(const Part &p, std::vector<Rank> &rk)
{
    std::vector<mpfft_copy> plan;
    exchange_plan(p, MPFFT_XCHG_COL_TO_ROW, plan);
    int rc;
    for (int d = 0; d < p.world; ++d) {
        SETDEV(rk[d]);
        for (int op = 0; op < 2; ++op) {
            for (int s = 0; s < p.world; ++s)
                if ((rc = wait(rk, d, true, s, op ? EV_MAIN : EV_A))) return rc;
            for (const mpfft_copy &c : plan)
                if (c.dst == d && c.op == op && (rc = queue_copy(rk, c, true, "xchg1"))) return rc;
        }
        if ((rc = rec(rk, d, EV_X, true))) return rc;
    }
    for (int d = 0; d < p.world; ++d) {   // senders' compute streams must not run ahead of the pulls
        SETDEV(rk[d]);
        for (int s = 0; s < p.world; ++s)
            if ((rc = wait(rk, d, false, s, EV_X))) return rc;
        if ((rc = rec(rk, d, EV_MAIN))) return rc;
    }
    return MPFFT_OK;
}

// queue a set of copies (an exchange or the halo): each receiver waits for every sender's last
// event, then pulls; the events are re-recorded only after every receiver queued its waits
int run_copies(const Part &p, std::vector<Rank> &rk, const std::vector<mpfft_copy> &plan, const char *what)
{
    int rc;
    for (int d = 0; d < p.world; ++d) {
        SETDEV(rk[d]);
        for (int s = 0; s < p.world; ++s)
            if (s != d && (rc = wait(rk, d, false, s, EV_MAIN))) return rc;
        for (const mpfft_copy &c : plan)
            if (c.dst == d && (rc = queue_copy(rk, c, false, what))) return rc;
    }
    for (int d = 0; d < p.world; ++d) {
        SETDEV(rk[d]);
        if ((rc = rec(rk, d, EV_MAIN))) return rc;
    }
    return MPFFT_OK;
}

int stage_all(const Part &p, std::vector<Rank> &rk, int stage, unsigned long depth, unsigned long w,
              bool ev_a = false)
{
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        SETDEV(R);
        const mpfft_shard sh = desc(p, d, R, depth, w);
        int rc;
        if (work(d, false, shard_stage_name(stage)) && (rc = mpfft_shard_stage(stage, &sh, R.in[0], R.in[1], R.s)))
            return rc;
        if (stage == MPFFT_SHARD_POINTWISE && p.fused) {   // the product is in rowc: operand 0 from here on
            std::swap(R.row[0], R.rowc);
            if (p.world == 1) std::swap(R.col[0], R.colc);
        }
        if ((rc = rec(rk, d, ev_a ? EV_A : EV_MAIN))) return rc;
    }
    return MPFFT_OK;
}

// the halo: every sender packs its outgoing runs (one launch), every receiver pulls one block
// per sender after that sender's pack, and scatters the blocks that are not contiguous in its halo
int run_halo(const Part &p, std::vector<Rank> &rk, const std::vector<HaloRank> &hr)
{
    int rc;
    for (int s = 0; s < p.world; ++s) {
        Rank &S = rk[s];
        SETDEV(S);
        if (!hr[s].pack.empty() && work(s, false, "halo_pack")) {
            hipLaunchKernelGGL(k_copy_runs, dim3((unsigned)std::min<size_t>(hr[s].pack.size(), 4096)), dim3(256), 0, S.s,
                               (const Run *)S.d_pack, (long)hr[s].pack.size(), (const u64 *)S.col[0].dig, S.hsend);
            MCHK(hipGetLastError());
        }
        if ((rc = rec(rk, s, EV_MAIN))) return rc;
    }
    for (int d = 0; d < p.world; ++d) {
        Rank &D = rk[d];
        SETDEV(D);
        for (int s = 0; s < p.world; ++s) {
            const Rank &S = rk[s];
            const long n = hr[s].send_cnt[d];
            if (!n) continue;
            if (s != d && (rc = wait(rk, d, false, s, EV_MAIN))) return rc;
            if (!copy_from(d, false, "halo", s)) continue;
            u64 *dp = hr[d].recv_halo[s] >= 0 ? D.halo + hr[d].recv_halo[s] : D.hstage + hr[d].recv_stage[s];
            const u64 *sp = S.hsend + hr[s].send_off[d];
            if (S.dev == D.dev) MCHK(hipMemcpyAsync(dp, sp, (size_t)n * 8, hipMemcpyDeviceToDevice, D.s));
            else MCHK(hipMemcpyPeerAsync(dp, D.dev, sp, S.dev, (size_t)n * 8, D.s));
        }
        if (!hr[d].scatter.empty() && work(d, false, "halo_scatter")) {
            hipLaunchKernelGGL(k_copy_runs, dim3((unsigned)std::min<size_t>(hr[d].scatter.size(), 4096)), dim3(256), 0,
                               D.s, (const Run *)D.d_scatter, (long)hr[d].scatter.size(), (const u64 *)D.hstage, D.halo);
            MCHK(hipGetLastError());
        }
    }
    for (int d = 0; d < p.world; ++d) {
        SETDEV(rk[d]);
        if ((rc = rec(rk, d, EV_MAIN))) return rc;
    }
    return MPFFT_OK;
}

// the whole multiply from every rank's operand slices (R.in) to its product stripes (R.out),
// queued on the ranks' streams with no host synchronisation.
//
// Event audit (tests/test_multi_schedule.py checks the recorded graph): an exchange's receivers
// wait for the senders' events before any of them is recorded again (run_copies, run_halo,
// run_exchange_fwd record in a separate loop or into a separate event); the stripe summaries are
// published in their own event evs, so phase 1 of rank d waits for phase 0 of every rank, never
// for another rank's phase 1; and a call starts, on every rank, after the end (evd) of every
// other rank's previous call -- its first writes to rank e's arrays (the split into the column
// arrays, exchange #1 into the row arrays) would otherwise overtake the previous call's pulls
// from them on the other ranks' streams (exchange #2 from e's row arrays, the halo send block,
// the summaries).
int run_ranks(const Part &p, std::vector<Rank> &rk, const std::vector<HaloRank> &halo, unsigned long depth,
              unsigned long w)
{
    int rc;
    for (int d = 0; d < p.world; ++d) {
        SETDEV(rk[d]);
        for (int e = 0; e < p.world; ++e)
            if (e != d && rk[e].done_rec && (rc = wait(rk, d, false, e, EV_DONE))) return rc;
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
    std::vector<mpfft_copy> plan;
    exchange_plan(p, MPFFT_XCHG_ROW_TO_COL, plan);
    if ((rc = run_copies(p, rk, plan, "xchg2"))) return rc;
    if ((rc = stage_all(p, rk, MPFFT_SHARD_INV_COLUMNS, depth, w))) return rc;
    if ((rc = run_halo(p, rk, halo))) return rc;
    // combine phase 0: every stripe with carry-in 0 and its (generate, propagate) summary
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        SETDEV(R);
        const mpfft_shard sh = desc(p, d, R, depth, w);
        if (work(d, false, "combine0") &&
            (rc = mpfft_shard_combine(&sh, 0, R.out, R.halo, R.sums, nullptr, R.tmp, R.tmp_bytes, R.s)))
            return rc;
        if ((rc = rec(rk, d, EV_SUM))) return rc;
    }
    // every rank's summaries to every rank (Tr pairs each), then phase 1: each rank scans the
    // stripes below each of its own on the device and adds the carry.  The pulls wait on evs
    // (phase 0), which no rank re-records in this loop: phase 1 runs on all ranks at once
    // (waiting on ev, re-recorded after each rank's phase 1 here, chained them 0 -> 1 -> ...)
    const size_t sb = (size_t)p.Tr * 2 * sizeof(int);
    for (int d = 0; d < p.world; ++d) {
        Rank &R = rk[d];
        SETDEV(R);
        for (int e = 0; e < p.world; ++e) {
            const Rank &E = rk[e];
            if (e != d && (rc = wait(rk, d, false, e, EV_SUM))) return rc;
            if (!copy_from(d, false, "sums", e)) continue;
            int *dp = R.sums_all + (size_t)e * p.Tr * 2;
            if (E.dev == R.dev) MCHK(hipMemcpyAsync(dp, E.sums, sb, hipMemcpyDeviceToDevice, R.s));
            else MCHK(hipMemcpyPeerAsync(dp, R.dev, E.sums, E.dev, sb, R.s));
        }
        const mpfft_shard sh = desc(p, d, R, depth, w);
        if (work(d, false, "combine1") &&
            (rc = mpfft_shard_combine(&sh, 1, R.out, R.halo, R.sums, R.sums_all, R.tmp, R.tmp_bytes, R.s)))
            return rc;
        if ((rc = rec(rk, d, EV_MAIN))) return rc;
        if ((rc = rec(rk, d, EV_DONE))) return rc;
        R.done_rec = true;
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

// the context for this device list (buffers set up for partition p)
int prepare(Ctx &X, const Part &p, const std::vector<int> &devs, bool host)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return MPFFT_ENODEV;
    for (int d : devs)
        if (d < 0 || d >= ndev) return MPFFT_ENODEV;
    if (X.devs != devs) {
        drain(X.ranks);
        for (Rank &R : X.ranks) free_rank(R);
        X.ranks.assign(devs.size(), Rank());
        for (size_t g = 0; g < devs.size(); ++g) X.ranks[g].dev = devs[g];
        X.devs = devs;
        enable_peers(devs);
    }
    const std::vector<long> key = part_key(p);
    if (X.key != key) {
        halo_xfer(p, X.halo);
        X.key = key;
    }
    // a rank whose buffers grow frees its old allocation: other ranks' streams (other devices)
    // may still be pulling from it -- exchange #2 from its row arrays, the halo send block, the
    // summaries -- after the previous device-resident call, which returns without a host sync
    bool grows = false;
    for (int d = 0; d < p.world; ++d) {
        size_t hb = 0;
        const size_t need = rank_need(p, d, host, X.halo[d], &hb);
        if (X.ranks[d].mem_bytes < need || X.ranks[d].host_bytes < hb) grows = true;
    }
    if (grows) drain(X.ranks);
    for (int d = 0; d < p.world; ++d) {
        int rc = setup_rank(p, d, X.ranks[d], host, X.halo[d]);
        if (rc) return rc;
    }
    return MPFFT_OK;
}

int mul_multi_locked(Ctx &X, uint64_t *r1, const uint64_t *i1, long n1, const uint64_t *i2, long n2,
                     unsigned long depth, unsigned long w, const std::vector<int> &devs)
{
    Part p;
    const int G = (int)devs.size();
    int rc = partition(p, n1, n2, depth, w, G);
    if (rc) return rc;
    if ((rc = prepare(X, p, devs, true))) return rc;
    std::vector<Rank> &rk = X.ranks;

    // operands in: the whole operands straight from the caller's arrays when every rank
    // computes every column block (replicated), else each rank's slices packed into its pinned
    // staging; one host thread per rank
    std::vector<int> trc(G, MPFFT_OK);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < G; ++d)
            th.emplace_back([&, d] {
                Rank &R = rk[d];
                if (hipSetDevice(R.dev) != hipSuccess) { trc[d] = MPFFT_EHIP; return; }
                if (p.rep) {
                    if (hipMemcpyAsync(R.src[0], i1, (size_t)n1 * 8, hipMemcpyHostToDevice, R.s) != hipSuccess ||
                        hipMemcpyAsync(R.src[1], i2, (size_t)n2 * 8, hipMemcpyHostToDevice, R.s) != hipSuccess)
                        trc[d] = MPFFT_EHIP;
                    return;
                }
                const long sl = p.src_limbs();
                pack_slices(p, d, i1, n1, R.host);
                pack_slices(p, d, i2, n2, R.host + sl);
                if (hipMemcpyAsync(R.src[0], R.host, (size_t)sl * 8, hipMemcpyHostToDevice, R.s) != hipSuccess ||
                    hipMemcpyAsync(R.src[1], R.host + sl, (size_t)sl * 8, hipMemcpyHostToDevice, R.s) != hipSuccess)
                    trc[d] = MPFFT_EHIP;
            });
        for (auto &t : th) t.join();
        for (int d = 0; d < G; ++d)
            if (trc[d]) return trc[d];
    }
    for (int d = 0; d < G; ++d) {
        rk[d].in[0] = rk[d].src[0];
        rk[d].in[1] = rk[d].src[1];
        rk[d].whole = p.rep;
        rk[d].out = rk[d].r;
    }
    rc = run_ranks(p, rk, X.halo, depth, w);
    for (int d = 0; d < G; ++d) rk[d].whole = false;
    if (rc) return rc;
    // product stripes out: per rank one D2H of its stripe buffer into its pinned staging, then
    // the stripes copied into their places in r1 (one host thread per rank)
    {
        std::vector<std::thread> th;
        for (int d = 0; d < G; ++d)
            th.emplace_back([&, d] {
                Rank &R = rk[d];
                if (hipSetDevice(R.dev) != hipSuccess ||
                    hipMemcpyAsync(R.host, R.r, (size_t)p.Tr * p.SL * 8, hipMemcpyDeviceToHost, R.s) != hipSuccess ||
                    hipStreamSynchronize(R.s) != hipSuccess) {
                    trc[d] = MPFFT_EHIP;
                    return;
                }
                for (long j = 0; j < p.Tr; ++j) {
                    const long s = j * G + d, cnt = p.ms[s + 1] - p.ms[s];
                    if (cnt > 0) memcpy(r1 + p.ms[s], R.host + j * p.SL, (size_t)cnt * 8);
                }
            });
        for (auto &t : th) t.join();
        for (int d = 0; d < G; ++d)
            if (trc[d]) return trc[d];
    }
    return MPFFT_OK;
}

int mul_multi_device_locked(Ctx &X, long n1, long n2, unsigned long depth, unsigned long w,
                            const std::vector<int> &devs, const uint64_t *const *d_src1,
                            const uint64_t *const *d_src2, uint64_t *const *d_r, void *const *streams)
{
    Part p;
    const int G = (int)devs.size();
    int rc = partition(p, n1, n2, depth, w, G);
    if (rc) return rc;
    if (!d_src1 || !d_src2 || !d_r) return MPFFT_EINVAL;
    if ((rc = prepare(X, p, devs, false))) return rc;
    std::vector<Rank> &rk = X.ranks;
    for (int d = 0; d < G; ++d) {
        Rank &R = rk[d];
        if (!d_src1[d] || !d_src2[d] || !d_r[d]) return MPFFT_EINVAL;
        R.in[0] = d_src1[d];
        R.in[1] = d_src2[d];
        R.out = d_r[d];
        if (streams && streams[d]) {   // after the caller's work on its stream
            MCHK(hipSetDevice(R.dev));
            MCHK(hipEventRecord(R.ev, (hipStream_t)streams[d]));
            MCHK(hipStreamWaitEvent(R.s, R.ev, 0));
        }
    }
    if ((rc = run_ranks(p, rk, X.halo, depth, w))) return rc;
    for (int d = 0; d < G; ++d) {
        Rank &R = rk[d];
        MCHK(hipSetDevice(R.dev));
        if (streams && streams[d]) {   // the caller's stream continues after the product
            MCHK(hipEventRecord(R.ev, R.s));
            MCHK(hipStreamWaitEvent((hipStream_t)streams[d], R.ev, 0));
        } else {
            MCHK(hipStreamSynchronize(R.s));
        }
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

// a device list every id of which exists (else the policy stays off: products run on the
// calling thread's device)
bool devices_exist(const std::vector<int> &v)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    for (int d : v)
        if (d < 0 || d >= ndev) return false;
    return true;
}

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
    if (v.size() > 1 && devices_exist(v)) g_pol.devs = v;
}

}  // namespace

// used by mpfft_mul_ex (mpfft.hip): the device list the policy picks for this product, if any
int mpfft_multi_policy(long n1, long n2, unsigned long depth, unsigned long w, std::vector<int> &devs)
{
    long min_l;
    {
        std::lock_guard<std::mutex> lk(g_pol.mu);
        policy_init_locked();
        if (g_pol.devs.size() < 2) return 0;
        devs = g_pol.devs;
        min_l = g_pol.min_l;
    }
    long info[10];
    if (mpfft_plan_info(n1, n2, depth, w, info) || info[1] < min_l) return 0;
    Part p;
    return partition(p, n1, n2, depth, w, (int)devs.size()) == MPFFT_OK ? (int)devs.size() : 0;
}

namespace {
// leave no work queued behind a failed call: compute and exchange streams of every rank
int finish(Ctx &X, int rc, int cur)
{
    if (rc) drain(X.ranks);
    (void)hipSetDevice(cur);
    return rc;
}
}  // namespace

extern "C" {

int mpfft_shard_partition(long n1, long n2, unsigned long depth, unsigned long w, int world, long *rows, long *info)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return rc;
    for (int d = 0; d <= world; ++d) rows[d] = p.rows[d];
    info[0] = p.C;
    info[1] = p.chunk;
    info[2] = p.H;
    info[3] = p.Tr;
    info[4] = p.fused ? 1 : 0;
    info[5] = p.SL;
    info[6] = p.S;
    return MPFFT_OK;
}

long mpfft_shard_stripes(long n1, long n2, unsigned long depth, unsigned long w, int world, long *ms, long cap)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return -rc;
    if (ms) {
        if (cap < p.S + 1) return -MPFFT_EINVAL;
        memcpy(ms, p.ms.data(), (size_t)(p.S + 1) * sizeof(long));
    }
    return p.S + 1;
}

static long copy_out(const std::vector<mpfft_copy> &v, mpfft_copy *out, long cap)
{
    if (out) {
        if (cap < (long)v.size()) return -MPFFT_EINVAL;
        memcpy(out, v.data(), v.size() * sizeof(mpfft_copy));
    }
    return (long)v.size();
}

long mpfft_shard_exchange_plan(long n1, long n2, unsigned long depth, unsigned long w, int world, int which,
                               mpfft_copy *out, long cap)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return -rc;
    if (which != MPFFT_XCHG_COL_TO_ROW && which != MPFFT_XCHG_ROW_TO_COL) return -MPFFT_EINVAL;
    std::vector<mpfft_copy> v;
    exchange_plan(p, which, v);
    return copy_out(v, out, cap);
}

long mpfft_shard_halo_plan(long n1, long n2, unsigned long depth, unsigned long w, int world, mpfft_copy *out,
                           long cap)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return -rc;
    std::vector<mpfft_copy> v;
    halo_plan(p, v);
    return copy_out(v, out, cap);
}

long mpfft_shard_src_limbs(long n1, long n2, unsigned long depth, unsigned long w, int world)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    return rc ? -rc : p.src_limbs();
}

int mpfft_shard_pack(long n1, long n2, unsigned long depth, unsigned long w, int world, int rank, const uint64_t *a,
                     long na, uint64_t *out)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return rc;
    if (rank < 0 || rank >= world || !a || !out || na < 0) return MPFFT_EINVAL;
    pack_slices(p, rank, a, na, out);
    return MPFFT_OK;
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
    return finish(g_ctx, mul_multi_locked(g_ctx, r1, i1, n1, i2, n2, depth, w, devs), cur);
}

int mpfft_mul_multi_device(long n1, long n2, unsigned long depth, unsigned long w, int ngpus, const int *devices,
                           const uint64_t *const *d_src1, const uint64_t *const *d_src2, uint64_t *const *d_r,
                           void *const *streams)
{
    if (ngpus < 1) return MPFFT_EINVAL;
    std::vector<int> devs(ngpus);
    for (int g = 0; g < ngpus; ++g) devs[g] = devices ? devices[g] : g;
    int cur = 0;
    (void)hipGetDevice(&cur);
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    (void)hipGetLastError();
    return finish(g_ctx, mul_multi_device_locked(g_ctx, n1, n2, depth, w, devs, d_src1, d_src2, d_r, streams), cur);
}

int mpfft_multi_release(void)
{
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    drain(g_ctx.ranks);
    for (Rank &R : g_ctx.ranks) free_rank(R);
    g_ctx.ranks.clear();
    g_ctx.devs.clear();
    (void)hipSetDevice(cur);
    return MPFFT_OK;
}

long mpfft_multi_schedule(long n1, long n2, unsigned long depth, unsigned long w, int world, int calls, char *buf,
                          size_t len)
{
    Part p;
    int rc = partition(p, n1, n2, depth, w, world);
    if (rc) return -rc;
    if (calls < 1) return -MPFFT_EINVAL;
    std::vector<Rank> rk(world);
    std::vector<HaloRank> hr;
    halo_xfer(p, hr);
    Sched sc;
    sc.dry = true;
    g_sched = &sc;
    for (int k = 0; k < calls && !rc; ++k) {
        if (k) sched_line("N");
        rc = run_ranks(p, rk, hr, depth, w);
    }
    g_sched = nullptr;
    if (rc) return -rc;
    if (buf && len) {
        const size_t n = std::min(len - 1, sc.log.size());
        memcpy(buf, sc.log.data(), n);
        buf[n] = 0;
    }
    return (long)sc.log.size() + 1;
}

int mpfft_set_devices(int ngpus, const int *devices, long min_l)
{
    std::vector<int> v;
    if (ngpus > 1)
        for (int g = 0; g < ngpus; ++g) v.push_back(devices ? devices[g] : g);
    if (!v.empty() && !devices_exist(v)) return MPFFT_ENODEV;
    std::lock_guard<std::mutex> lk(g_pol.mu);
    g_pol.init = true;   // an explicit choice overrides MPFFT_DEVICES
    g_pol.devs = v;
    g_pol.min_l = min_l > 0 ? min_l : 1024;
    return MPFFT_OK;
}

}  // extern "C"
