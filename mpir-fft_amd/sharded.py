"""Column-sharded new_mpn_mul over the ranks of a torch.distributed group
(BASELINE configs[4]: "MFA columns sharded 8-way with RCCL all-to-all over xGMI
between the column and row passes").

The matrix Fourier algorithm's column transforms are independent per column
(/root/reference/mul_fft.c:2374-2390) and its row transforms, pointwise products
and row inverses are independent per row (:2392-2408, :3244-3253, :2942-2957).
So:

  rank g owns columns [g*C, (g+1)*C), C = NC / world     (column layout)
  1. split + forward column passes of both operands on the owned columns
  2. exchange #1: rows [r_d, r_{d+1}) of every column block -> rank d
  3. twiddle + forward row passes, pointwise, inverse row passes on owned rows
  4. exchange #2: the rows go back to their column owners
  5. truncated inverse column transform + scaling on the owned columns
  6. halo: for each row position, the H coefficients before the rank's C columns
  7. combine in the column layout: the rank's C columns of row position j are the C
     consecutive coefficients [(j world + g) C, + C) -- product stripe j world + g, a
     contiguous bit range -- combined with carry-in 0; an all-gather of every stripe's
     (generate, propagate) pair; each stripe's carry-in added on the device

The product ends up striped: rank g holds stripes j world + g (mpfft_shard_stripes gives
their limb ranges; mpfft.assemble_stripes puts them in order).  Exchanges are batches of
point-to-point send/recv (RCCL over xGMI on GPUs, gloo on CPU for the tests); no
all-reduce is used.  #1 moves both operands, #2 the product once; the product never
goes back to row owners (the reference's TODO:53-59: combine in place, for locality).
"""
import os

import numpy as np


XCHG_COL_TO_ROW, XCHG_ROW_TO_COL = 1, 2   # include/mpfft.h MPFFT_XCHG_*


def cb_words(l):
    return 2 * ((l + 63) // 64)


class ShardPlan:
    """Partition of one multiply over `world` ranks: the library's own partition
    (mpfft_shard_partition, csrc/multi.hip), so this harness and the one-process C driver
    mpfft_mul_multi shard identically; tests/test_sharded_cpu.py restates it independently."""

    def __init__(self, mp, n1, n2, depth, w, world):
        P = mp.plan_info(n1, n2, depth, w)
        self.mp = mp
        self.n1, self.n2, self.depth, self.w, self.world = n1, n2, depth, w, world
        self.n, self.l, self.NC, self.NR = P["n"], P["l"], P["NC"], P["NR"]
        self.T, self.bits1 = P["trunc"], P["bits1"]
        self.N = self.n * w
        self.len = P["j1"] + P["j2"] - 1
        self.Tr = self.T // self.NC
        self.total = n1 + n2
        self.cbw = cb_words(self.l)
        if self.NC % world or world & (world - 1):
            raise ValueError(f"world={world} must be a power of two dividing NC={self.NC}")
        try:
            part = mp.shard_partition(n1, n2, depth, w, world)
        except mp.MpfftError as e:
            raise ValueError(f"world={world}: too many ranks for this size ({e})") from None
        self.C = part["C"]                 # columns per rank (= column block of the row layout)
        self.rows = part["rows"]           # rank d owns live rows [rows[d], rows[d+1])
        self.H = part["H"]                 # halo: coefficients before a stripe that reach its limbs
        self.SL, self.S = part["SL"], part["S"]   # limbs per stripe at most; stripes (world Tr)
        self.ms = part["ms"]               # stripe s = j world + g: product limbs [ms[s], ms[s+1])
        # operand column slices (fused split reads them through SrcSlice, coeff.hpp): for
        # each live position p < Tr, `chunk` limbs from floor((p NC + c0) bits1 / 64) on
        self.chunk = part["chunk"]
        self._xplans = {}

    def exchange_plan(self, which):
        """the copies of exchange `which` (mp.XCHG_*), from the library (mpfft_shard_exchange_plan)"""
        if which not in self._xplans:
            self._xplans[which] = self.mp.shard_exchange_plan(self.n1, self.n2, self.depth, self.w, self.world,
                                                              which)
        return self._xplans[which]

    def halo_plan(self):
        """the halo copies before the combine (mpfft_shard_halo_plan): column layout -> halo,
        offsets and counts in limbs"""
        if "halo" not in self._xplans:
            self._xplans["halo"] = self.mp.shard_halo_plan(self.n1, self.n2, self.depth, self.w, self.world)
        return self._xplans["halo"]

    def slice_start(self, p, d):
        return ((p * self.NC + d * self.C) * self.bits1) // 64

    def slice_operand(self, a, d):
        """rank d's column slice of operand a (uint64 limbs): Tr chunks of `chunk` limbs."""
        out = np.zeros(self.Tr * self.chunk, dtype=np.uint64)
        for p in range(self.Tr):
            s0 = self.slice_start(p, d)
            if s0 >= len(a):
                break
            seg = a[s0: s0 + self.chunk]
            out[p * self.chunk: p * self.chunk + len(seg)] = seg
        return out

    def rcount(self, d):
        return self.rows[d + 1] - self.rows[d]

    def assemble(self, stripes):
        """the product (uint64 limbs) from every rank's stripe buffer (rank order, numpy uint64)"""
        return self.mp.assemble_stripes({"ms": self.ms, "SL": self.SL}, self.world, stripes)

    def col_slots(self):
        return self.NR * self.C

    def row_slots(self, d):
        return self.rcount(d) * self.NC


class ShardedMul:
    """One rank's part.  `backend` runs the stages on this rank's buffers,
    `comm` moves them (both duck-typed; see GpuBackend / TorchComm)."""

    # world > 1: the row phase in this many row chunks (exchange #2 overlapped); MPFFT_ROW_CHUNKS
    # overrides (diagnostics / A/B)
    row_chunks = int(os.environ.get("MPFFT_ROW_CHUNKS", "4"))

    def __init__(self, plan, rank, backend, comm, sliced=True, replicate=False):
        self.p, self.rank, self.be, self.comm = plan, rank, backend, comm
        self.sliced = sliced          # run() gets this rank's operand slices (ShardPlan.slice_operand)
        # replicate: every rank computes every column block's forward columns from the whole
        # operands and keeps its own rows of each, so exchange #1 moves nothing (see replicates)
        if replicate and sliced:
            raise ValueError("replicated forward columns need the whole operands (sliced=False)")
        self.replicate = replicate
        p = plan
        self.col = [backend.alloc_coeffs(p.col_slots()) for _ in range(2)]
        if p.world == 1:
            # one rank: the row layout (ccb = C = NC, rows [0, Tr)) is the column layout's first
            # Tr NC slots, so the row arrays are views of the column arrays and the exchanges
            # find nothing to move (no stage reads one layout while writing the other)
            self.row = [{f: c[f][: p.row_slots(rank) * backend.width(f, p)] for f in c} for c in self.col]
        else:
            self.row = [backend.alloc_coeffs(p.row_slots(rank)) for _ in range(2)]
        # the row DIF's last level fused into the pointwise, as on one GPU: the product lands in
        # a third row array, which then serves as operand 0's row array (swapped after the stage).
        # At world 1 that array is a view of a third column-layout array, swapped together with
        # col[0], so the row arrays stay views of the column arrays on every run.
        self._hidx = None   # the halo plan as index tensors (_halo_index)
        self.fused = bool(getattr(backend, "row_fused", lambda: False)())
        self.colc = None
        if self.fused and p.world == 1:
            self.colc = backend.alloc_coeffs(p.col_slots())
            self.rowc = {f: self.colc[f][: p.row_slots(rank) * backend.width(f, p)] for f in self.colc}
        else:
            self.rowc = backend.alloc_coeffs(p.row_slots(rank)) if self.fused else None

    @staticmethod
    def replicates(world):
        """the forward-column policy for `world` ranks: replicated at world 2, where exchange
        #1 is one xGMI link carrying, each way, the other rank's half of both operands' column
        blocks (C4: 2 x 1.25 GB, ≈ 33 ms at 76 GB/s) and the second column block costs one
        more column phase of HBM-bound passes (C4: ≈ 9 ms); at world 4 the exchange spreads
        over three links (≈ 0.63 GB per link and direction, ≈ 8 ms) and replication would cost
        three more blocks (≈ 14 ms), so the columns stay sharded.
        MPFFT_REPLICATE_COLUMNS=0/1 overrides (A/B)."""
        env = os.environ.get("MPFFT_REPLICATE_COLUMNS")
        if env is not None:
            return env == "1" and world > 1
        return world == 2

    def shard_desc(self):
        p, d = self.p, self.rank
        return dict(n1=p.n1, n2=p.n2, depth=p.depth, w=p.w, c0=d * p.C, ccount=p.C,
                    r0=p.rows[d], rcount=p.rcount(d), ccb=p.C, col=list(self.col), row=list(self.row),
                    src_chunk=p.chunk if self.sliced else 0, rowc=self.rowc)

    # one exchange from the library's copy plan (the same copies mpfft_mul_multi issues as
    # peer DMA): #1 column layout rows [r_d, r_{d+1}) -> rank d's row layout block (both
    # operands), #2 back (the product), #3 the canonical limbs again.  Every (operand, field)
    # is one (send views by peer, recv views by peer) entry; all go in one batch of
    # point-to-point ops
    _FIELDS = ("dig", "cb", "top")

    def _exchange(self, which, op=None, wait=True, chunk=None):
        """op: only that operand's copies; wait=False: returns the pending transfers
        (comm.wait them later), so compute queued meanwhile overlaps the exchange.
        chunk = (i, R): exchange #2 for row chunk i of R of every row-layout rank (rows are
        contiguous, C slots each, on both sides of every copy)."""
        p, me = self.p, self.rank
        W = p.world

        def arr(layout, k):
            return self.row[k] if layout else self.col[k]
        groups = {}
        for c in p.exchange_plan(which):
            if me not in (c["src"], c["dst"]) or (op is not None and c["op"] != op):
                continue
            if chunk is not None:   # this chunk's rows of the row-layout rank (the sender of #2)
                d = c["src"] if which == XCHG_ROW_TO_COL else c["dst"]
                rc_d = p.rcount(d)
                a_, b_ = chunk_rows(rc_d, *chunk)
                per = c["count"] // rc_d          # C slots x field width per row
                c = dict(c, src_off=c["src_off"] + a_ * per, dst_off=c["dst_off"] + a_ * per, count=(b_ - a_) * per)
                if not c["count"]:
                    continue
            f = self._FIELDS[c["field"]]
            send, recv = groups.setdefault((c["op"], c["field"]), ([None] * W, [None] * W))
            if c["src"] == me:
                send[c["dst"]] = arr(c["src_layout"], c["op"])[f][c["src_off"]: c["src_off"] + c["count"]]
            if c["dst"] == me:
                recv[c["src"]] = arr(c["dst_layout"], c["op"])[f][c["dst_off"]: c["dst_off"] + c["count"]]
        plan = []
        for (op, fi) in sorted(groups):
            send, recv = groups[(op, fi)]
            empty = self.col[op][self._FIELDS[fi]][:0]
            plan.append(([v if v is not None else empty for v in send], [v if v is not None else empty for v in recv]))
        return self.comm.exchange(plan, wait=wait)

    def _halo_index(self):
        """the halo plan as coefficient indices, built once per job: per receiver the column-layout
        slots this rank sends (in plan order), per sender where its block lands in this rank's
        halo -- a contiguous range (always when H <= C) or halo slots to scatter to"""
        if self._hidx is None:
            import torch
            p, me, W, l = self.p, self.rank, self.p.world, self.p.l
            send, runs = [[] for _ in range(W)], [[] for _ in range(W)]
            for c in p.halo_plan():
                if c["src"] == me:
                    send[c["dst"]].extend(range(c["src_off"] // l, (c["src_off"] + c["count"]) // l))
                if c["dst"] == me:
                    runs[c["src"]].append((c["dst_off"] // l, c["count"] // l))
            dev = self.col[0]["dig"].device
            sidx = [torch.tensor(ix, dtype=torch.int64, device=dev) if ix else None for ix in send]
            recv = []
            for d in range(W):
                r = runs[d]
                if not r:
                    recv.append(None)
                elif all(r[i][0] + r[i][1] == r[i + 1][0] for i in range(len(r) - 1)):
                    recv.append((r[0][0], sum(n for _, n in r), None))      # straight into the halo
                else:
                    ix = [s0 + k for s0, n in r for k in range(n)]
                    recv.append((0, len(ix), torch.tensor(ix, dtype=torch.int64, device=dev)))
            self._hidx = (sidx, recv)
        return self._hidx

    def _halo(self, halo):
        """the H coefficients before each of this rank's stripes into `halo` (Tr H l limbs): one
        gathered message per peer (an index_select over the column layout's coefficients)"""
        p, l = self.p, self.p.l
        sidx, ridx = self._halo_index()
        col = self.col[0]["dig"].view(-1, l)
        empty = self.col[0]["dig"][:0]
        send = [col.index_select(0, ix).view(-1) if ix is not None else empty for ix in sidx]
        recv, scatter = [], []
        for r in ridx:
            if r is None:
                recv.append(empty)
            elif r[2] is None:
                recv.append(halo[r[0] * l: (r[0] + r[1]) * l])
            else:
                buf = halo.new_empty(r[1] * l)
                recv.append(buf)
                scatter.append((buf, r[2]))
        self.comm.exchange([(send, recv)], wait=True)
        for buf, ix in scatter:
            halo.view(-1, l).index_copy_(0, ix, buf.view(-1, l))

    def run(self, i1, i2, mark=None):
        """i1, i2: this rank's operand column slices (ShardPlan.slice_operand; the full
        operands when sliced=False), backend arrays.  Returns this rank's product stripes
        (Tr SL limbs: stripe j world + rank at j SL, ShardPlan.ms gives their limb ranges).
        mark(name), when given, is called after each phase (bench.py's per-phase events)."""
        p, be, sh = self.p, self.be, self.shard_desc()
        chunked_ok = mark is None
        mark = mark or (lambda name: None)
        if self.replicate:
            # every column block's forward columns here in turn (the column arrays are scratch
            # for the block being computed), then this rank's rows of that block copied to its
            # row layout: exchange #1's copies with every source rank played locally
            recv = [c for c in p.exchange_plan(XCHG_COL_TO_ROW) if c["dst"] == self.rank]
            for d in range(p.world):
                be.stage("fwd_columns_own", dict(sh, c0=d * p.C), i1, i2)   # this rank's rows of block d
                for c in recv:
                    if c["src"] == d:
                        f = self._FIELDS[c["field"]]
                        src = (self.row if c["src_layout"] else self.col)[c["op"]][f]
                        dst = (self.row if c["dst_layout"] else self.col)[c["op"]][f]
                        dst[c["dst_off"]: c["dst_off"] + c["count"]].copy_(src[c["src_off"]: c["src_off"] + c["count"]])
            mark("fwd_columns")
        elif getattr(be, "split_columns", False):
            # operand 1's exchange in flight while operand 2's column passes run (on RCCL: the
            # transfers go on the communicator's stream, queued behind operand 1's passes only)
            be.stage("fwd_columns_a", sh, i1, i2)
            pend1 = self._exchange(XCHG_COL_TO_ROW, op=0, wait=False)
            be.stage("fwd_columns_b", sh, i1, i2)
            mark("fwd_columns")
            pend1 += self._exchange(XCHG_COL_TO_ROW, op=1, wait=False)
            self.comm.wait(pend1)          # exchange #1 complete before the row passes
        else:
            be.stage("fwd_columns", sh, i1, i2)
            mark("fwd_columns")
            self._exchange(XCHG_COL_TO_ROW)
        mark("exchange1")
        # (a run with per-phase marks -- bench.py's phase breakdown -- keeps the phases whole)
        R = self.row_chunks if (p.world > 1 and hasattr(be, "stage_rows") and chunked_ok) else 1
        if R > 1:
            # the row phase in R row chunks, each chunk's exchange #2 in flight while the next
            # computes (chunk i of every rank: chunk_rows; the senders' chunking is known to all)
            sh_fwd = sh      # (its own copies of the array lists: the swap below leaves it as it is)
            if self.fused:
                self.row[0], self.rowc = self.rowc, self.row[0]
            sh_inv = self.shard_desc()   # operand 0's row array = the product
            pend2 = []
            for i in range(R):
                lo, hi = chunk_rows(p.rcount(self.rank), i, R)
                be.stage_rows("fwd_rows", sh_fwd, lo, hi)
                be.stage_rows("pointwise", sh_fwd, lo, hi)
                be.stage_rows("inv_rows", sh_inv, lo, hi)
                pend2 += self._exchange(XCHG_ROW_TO_COL, wait=False, chunk=(i, R))
            mark("inv_rows")
            sh = sh_inv
        else:
            be.stage("fwd_rows", sh, i1, i2)
            mark("fwd_rows")
            be.stage("pointwise", sh, i1, i2)
            mark("pointwise")
            if self.fused:   # the product is in rowc: it becomes operand 0's row array
                self.row[0], self.rowc = self.rowc, self.row[0]
                if self.colc is not None:   # world 1: and its column array operand 0's
                    self.col[0], self.colc = self.colc, self.col[0]
                sh = self.shard_desc()
            be.stage("inv_rows", sh, i1, i2)
            mark("inv_rows")
            pend2 = self._exchange(XCHG_ROW_TO_COL, wait=False)
        self.comm.wait(pend2)          # exchange #2 complete before the inverse columns
        mark("exchange2")
        be.stage("inv_columns", sh, i1, i2)
        mark("inv_columns")
        # combine in the column layout: the H coefficients before each stripe, every stripe
        # with carry-in 0, every rank's stripe summaries, each stripe's carry-in
        halo = be.halo_buffer()
        self._halo(halo)
        mark("exchange_halo")
        r, sums = be.combine(sh, 0, halo)
        sums_all = self.comm.all_gather(sums)
        be.combine(sh, 1, halo, sums_all)
        mark("combine")
        return r


def chunk_rows(rcount, i, R):
    """local rows of chunk i of R of a rank holding rcount rows"""
    return rcount * i // R, rcount * (i + 1) // R


def _same_view(a, b):
    """a and b are the same elements of the same buffer (a local exchange with nothing to move)."""
    if hasattr(a, "data_ptr"):
        return a.data_ptr() == b.data_ptr() and a.numel() == b.numel() and a.dtype == b.dtype
    return a is b or (getattr(a, "base", None) is not None and a.__array_interface__["data"] == b.__array_interface__["data"]
                      and a.shape == b.shape)


def torch_empty_like_cpu(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


class TorchComm:
    """torch.distributed exchanges.  host_staging=True routes GPU tensors through the
    host (gloo on one GPU box / CPU tests); otherwise RCCL moves device buffers over xGMI."""

    def __init__(self, host_staging=False):
        import torch.distributed as dist
        self.dist = dist
        self.host = host_staging

    def all_to_all(self, out, inp, out_splits, in_splits):
        if self.host and out.is_cuda:
            o = out.cpu()
            self.dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
            out.copy_(o)
        else:
            self.dist.all_to_all_single(out, inp, out_splits, in_splits)

    def exchange(self, plan, wait=True):
        """plan: [(send views by peer, recv views by peer)]; one batch of isend/irecv for
        all of them (one RCCL group on GPUs), the rank's own views copied locally.
        wait=False (device buffers): returns the pending requests for wait(); host-staged
        exchanges always complete here."""
        me = self.dist.get_rank()
        ops, back = [], []
        for send, recv in plan:
            if not _same_view(recv[me], send[me]):
                recv[me].copy_(send[me])
            for d in range(len(send)):
                if d == me:
                    continue
                sv, rv = send[d], recv[d]
                if self.host and sv.is_cuda:
                    sv = sv.cpu()
                    rh = torch_empty_like_cpu(rv)
                    back.append((rv, rh))
                    rv = rh
                if sv.numel():
                    ops.append(self.dist.P2POp(self.dist.isend, sv.contiguous(), d))
                if rv.numel():
                    ops.append(self.dist.P2POp(self.dist.irecv, rv, d))
        reqs = self.dist.batch_isend_irecv(ops) if ops else []
        if wait or back:
            self.wait(reqs)
            reqs = []
        for dst, h in back:
            dst.copy_(h)
        return reqs

    @staticmethod
    def wait(reqs):
        for r in reqs:
            r.wait()

    def all_gather(self, t):
        import torch
        src = t.cpu() if (self.host and t.is_cuda) else t
        bufs = [torch.empty_like(src) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(bufs, src.contiguous())
        return bufs


class GpuBackend:
    """Stages through libmpfft's mpfft_shard_* C ABI on torch device buffers."""

    def __init__(self, mp, plan, device, stream=None):
        import torch
        self.mp, self.p, self.dev, self.torch = mp, plan, device, torch
        self.stream = stream
        self._tmp = None

    def width(self, field, p):
        return {"dig": p.l, "cb": p.cbw, "top": 1}[field]

    def row_fused(self):
        p = self.p
        return self.mp.shard_row_fused(p.n1, p.n2, p.depth, p.w, p.C)

    def alloc_coeffs(self, slots):
        t = self.torch
        p = self.p
        return {"dig": t.empty(slots * p.l, dtype=t.int64, device=self.dev),
                "cb": t.zeros(slots * p.cbw, dtype=t.int64, device=self.dev),
                "top": t.zeros(slots, dtype=t.int32, device=self.dev)}

    def _desc(self, sh):
        return self.mp.shard_desc(sh)

    split_columns = True   # per-operand forward column stages (exchange #1 overlaps operand 2's)

    def stage_rows(self, name, sh, lo, hi):
        """a row stage on local rows [lo, hi) (the chunked row phase)"""
        which = {"fwd_rows": 1, "pointwise": 2, "inv_rows": 3}[name]
        self.mp.shard_stage_rows(which, self._desc(sh), lo, hi, self.stream)

    def stage(self, name, sh, i1, i2):
        which = {"fwd_columns": 0, "fwd_rows": 1, "pointwise": 2, "inv_rows": 3, "inv_columns": 4,
                 "fwd_columns_a": 5, "fwd_columns_b": 6, "fwd_columns_own": 7}[name]
        self.mp.shard_stage(which, self._desc(sh), i1, i2, self.stream)

    def halo_buffer(self):
        p = self.p
        if getattr(self, "_halo_t", None) is None:
            self._halo_t = self.torch.zeros(p.Tr * p.H * p.l, dtype=self.torch.int64, device=self.dev)
        return self._halo_t

    def combine(self, sh, phase, halo, sums_all=None):
        """phase 0: (stripes, summaries) with carry-in 0; phase 1: each stripe's carry-in from
        every rank's summaries (a list, rank order)"""
        t, p = self.torch, self.p
        if self._tmp is None:
            nb = self.mp.shard_combine_tmp_bytes(p.n1, p.n2, p.depth, p.w, p.world)
            self._tmp = t.empty(max(nb, 1), dtype=t.uint8, device=self.dev)
            self._r = t.empty(p.Tr * p.SL, dtype=t.int64, device=self.dev)
            self._sums = t.zeros(2 * p.Tr, dtype=t.int32, device=self.dev)
        desc = self._desc(sh)
        if phase == 0:
            self.mp.shard_combine(desc, 0, self._r, halo, self._sums, None, self._tmp, self.stream)
            return self._r, self._sums
        allv = t.cat([x.to(self.dev) for x in sums_all])
        self.mp.shard_combine(desc, 1, self._r, halo, self._sums, allv, self._tmp, self.stream)
        return self._r


# algorithmic HBM bytes of one rank's phase (1/world of the whole multiply's)
def _phase_bytes(P, name, n1, n2, world):
    T, l = P["trunc"], P["l"]
    blk = 8 * l + 4
    whole = {"fwd_columns": 8 * (n1 + n2) + 2 * T * blk, "fwd_rows": 4 * T * blk, "pointwise": 3 * T * blk,
             "inv_rows": 2 * T * blk, "inv_columns": 4 * T * blk, "combine": T * blk + 8 * (n1 + n2)}
    return whole[name] / world if name in whole else None


def bench(args, cfg_name, cfg, rank, world, dev):
    """`bench.py --gpus N` (N > 1) / `--mode sharded`: one multiply of `cfg` split over
    all ranks (strong scaling).  Returns rank 0's JSON record (driver contract fields)."""
    import hashlib
    import json
    import os
    import time

    import torch
    import torch.distributed as dist
    import mpfft_loader
    mp = mpfft_loader.load()
    depth, w, nl = cfg
    plan = ShardPlan(mp, nl, nl, depth, w, world)
    a = mp.fill_random(nl, 0x1001)
    b = mp.fill_random(nl, 0x2002)
    rep = ShardedMul.replicates(world)
    if rep:   # replicated forward columns: the whole operands on every rank
        ha, hb = a, b
    else:     # only this rank's column slices of the operands travel to its GPU (1/world of each)
        ha = plan.slice_operand(a, rank)
        hb = plan.slice_operand(b, rank)
    del a, b
    da = torch.from_numpy(ha.view(np.int64)).to(dev)
    db = torch.from_numpy(hb.view(np.int64)).to(dev)
    be = GpuBackend(mp, plan, dev)
    rccl = world > 1 and dist.get_backend() == "nccl"
    comm = TorchComm(host_staging=(world > 1 and not rccl)) if world > 1 else _SoloComm()
    job = ShardedMul(plan, rank, be, comm, sliced=not rep, replicate=rep)

    def sync_all():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if rccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        job.run(da, db)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        limbs = job.run(da, db)
    sync_all()
    el = max_over_ranks(time.perf_counter() - t0)

    # per-phase device time of one more multiply: torch events on the current stream (the
    # library's kernels and the exchanges run there), max over ranks per phase
    evs = [("start", torch.cuda.Event(enable_timing=True))]
    evs[0][1].record()

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append((name, e))
    job.run(da, db, mark=mark)
    sync_all()
    phase_ms = {evs[i][0]: max_over_ranks(evs[i - 1][1].elapsed_time(evs[i][1])) for i in range(1, len(evs))}
    P = mp.plan_info(nl, nl, depth, w)
    comp = {k: v for k, v in phase_ms.items() if not k.startswith("exchange")}
    dname = max(comp, key=comp.get)
    dbytes = _phase_bytes(P, dname, nl, nl, world)
    # HBM traffic of the dominant phase's kernel from the committed one-GPU counter pass of the
    # same product (profiles/pmc_<cfg>.json, rocprofv3 --pmc, gfx950-corrected): a rank's
    # launch covers 1/world of the slots of the one-GPU launch
    traffic, tsrc = None, None
    kern = {"pointwise": "k_pwss"}.get(dname)
    if kern:
        try:
            pmc = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "profiles", f"pmc_{cfg_name}.json")))
            for name, rec in pmc.get("kernels", {}).items():
                if kern in name and rec.get("hbm_bytes_per_launch"):
                    traffic = rec["hbm_bytes_per_launch"] / world
                    tsrc = f"profiles/pmc_{cfg_name}.json ({name.split('(')[0]}, one-GPU launch) / world"
                    break
        except (OSError, ValueError):
            pass
    roof = {"bound": "hbm", "achieved": dbytes / (comp[dname] * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
            "frac": dbytes / (comp[dname] * 1e-3) / 8.0e12, "traffic": traffic, "traffic_source": tsrc,
            "stage": dname, "avg_ms": comp[dname], "alg_bytes_per_launch": dbytes,
            "note": "the slowest rank's dominant phase (all of its launches) vs one GPU's HBM peak; "
                    "algorithmic bytes = the phase's whole-multiply bytes / world"}

    # end to end from host operands: this rank's column slices H2D, the multiply, its stripes D2H
    sync_all()
    t1 = time.perf_counter()
    ea = torch.from_numpy(ha.view(np.int64)).to(dev)
    eb = torch.from_numpy(hb.view(np.int64)).to(dev)
    el2 = job.run(ea, eb)
    host_limbs = el2.cpu()
    sync_all()
    e2e_ms = max_over_ranks(time.perf_counter() - t1) * 1e3
    del ea, eb, host_limbs

    # exactness: rank 0 gathers every rank's stripes, puts them in order and hashes them
    exact = None
    if not getattr(args, "no_check", False):
        if rank == 0:
            parts = [limbs.cpu().numpy().view(np.uint64)]
            for d in range(1, world):
                buf = torch.empty(plan.Tr * plan.SL, dtype=torch.int64, device=dev if rccl else "cpu")
                dist.recv(buf, src=d)
                parts.append(buf.cpu().numpy().view(np.uint64))
            prod = plan.assemble(parts)
            h = hashlib.sha256(prod.tobytes())
            gp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                              "products.json")
            try:
                want = {c["name"]: c["sha256"] for c in json.load(open(gp))}.get(cfg_name)
                exact = h.hexdigest() == want if want else None
            except OSError:
                exact = None
        elif world > 1:
            dist.send(limbs if rccl else limbs.cpu(), dst=0)
    A = P["trunc"] * (P["l"] + 1) * 8
    balg = 8 * A + 32 * nl
    if world == 1:
        comm_label = "local exchanges (world 1)"
    elif rccl:
        comm_label = "RCCL over xGMI"
    else:
        comm_label = "gloo, host-staged (ranks sharing one GPU: a rehearsal, not a measurement)"
    return {"metric": "limbs/s for new_mpn_mul N×N-bit at 1/2/4/8 MI355X; % HBM roofline",
            "value": 2 * nl * args.steps / el, "unit": "limbs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (xoshiro256** limbs, seeds 0x1001/0x2002)",
            "config": {"workload": f"{cfg_name}: sharded new_mpn_mul depth={depth} w={w} n1=n2={nl} limbs "
                                   f"(l={P['l']}, NC x NR = {P['NC']} x {P['NR']}, trunc={P['trunc']})",
                       "parallelism": (f"MFA columns x{world}, " + (
                                "forward columns replicated (whole operands on every rank), exchange #1 local; "
                                "1 batched point-to-point exchange" if rep else
                                "operand column slices, 2 batched point-to-point exchanges") +
                                f" + per-stripe halo + summary all-gather, combine in the column layout ({comm_label})"),
                       "row_fused": job.fused},
            "roofline": roof,
            "phases_ms": phase_ms,
            "pipeline": {"b_alg_bytes": balg,
                         "hbm_frac_b_alg": balg / (el / args.steps) / (world * 8.0e12),
                         "note": "whole multiply vs the aggregate HBM roofline of the ranks (SURVEY 8d)"},
            "cpu_baseline": {"value": None, "unit": "limbs/s", "kind": "port",
                             "note": "timed on the N = 1 line only (rank 0, bounded sample: the bench contract); "
                                     "see BENCH_rNN.json cpu_baseline"},
            "e2e_host": {"ms": e2e_ms, "limbs_per_s": 2 * nl / (e2e_ms * 1e-3),
                         "note": "per rank: its operands (column slices, or whole when replicated) H2D, the multiply, its product stripes D2H "
                                 "(host slicing excluded); max over ranks"},
            "exact": exact}


class _SoloComm:
    """world == 1: exchanges are local copies."""

    def exchange(self, plan, wait=True):
        for send, recv in plan:
            if not _same_view(recv[0], send[0]):
                recv[0].copy_(send[0])
        return []

    @staticmethod
    def wait(reqs):
        pass

    def all_to_all(self, out, inp, out_splits, in_splits):
        out[: inp.numel()].copy_(inp)

    def all_gather(self, t):
        return [t]
