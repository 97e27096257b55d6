"""CPU stand-in for sharded.GpuBackend (tests only).

Implements every stage of the sharded pipeline with exact Python-int arithmetic
on the SAME per-rank buffer layouts (column layout / blocked row layout) that
the HIP kernels use, so a gloo world-size-2/4 run on CPU exercises the real
partitioning, the three all-to-all exchanges, the halo all-gather and the
cross-rank carry scan of mpir-fft_amd/sharded.py.  Stage semantics follow
SURVEY.md 8a (forward slot map, pointwise, truncated inverse); the inverse
column transform is a line-for-line port of the host recursion in
mpir-fft_amd/csrc/mpfft.hip (itft / itft1), so that recursion is also checked
here on CPU.
"""
import numpy as np
import torch

from helpers import log2, revbin


class MockBackend:
    def __init__(self, plan):
        self.p = plan
        p = plan
        self.mod = (1 << p.N) + 1
        self.lbR, self.lbC = log2(p.NR), log2(p.NC)

    # ---- storage -------------------------------------------------------
    def width(self, field, p):
        return {"dig": p.l, "cb": p.cbw, "top": 1}[field]

    def alloc_coeffs(self, slots):
        p = self.p
        return {"dig": torch.zeros(slots * p.l, dtype=torch.int64),
                "cb": torch.zeros(slots * p.cbw, dtype=torch.int64),
                "top": torch.zeros(slots, dtype=torch.int32)}

    def get(self, buf, slot):
        l = self.p.l
        limbs = buf["dig"][slot * l:(slot + 1) * l].numpy().view(np.uint64)
        v = int.from_bytes(limbs.tobytes(), "little") + int(buf["top"][slot]) * (1 << self.p.N)
        return v % self.mod

    def put(self, buf, slot, v):
        l, N = self.p.l, self.p.N
        v %= self.mod
        top = 1 if v == (1 << N) else 0
        lim = 0 if top else v
        arr = np.frombuffer(lim.to_bytes(8 * l, "little"), dtype=np.uint64).view(np.int64)
        buf["dig"][slot * l:(slot + 1) * l] = torch.from_numpy(arr.copy())
        buf["top"][slot] = top

    def pw(self, e):
        return pow(2, e % (2 * self.p.N), self.mod)

    # ---- layouts -------------------------------------------------------
    @staticmethod
    def col_slot(sh, pos, cl):
        return pos * sh["ccount"] + cl

    @staticmethod
    def row_slot(sh, pl, c):
        C = sh["ccb"]
        return (c // C) * sh["rcount"] * C + pl * C + (c % C)

    # ---- stages --------------------------------------------------------
    def stage(self, name, sh, i1, i2):
        getattr(self, "_" + name)(sh, i1, i2)

    split_columns = True   # per-operand forward column stages, as the GPU backend

    def _fwd_columns_a(self, sh, i1, i2):
        self._fwd_columns(sh, i1, i2, ops=(0,))

    def _fwd_columns_b(self, sh, i1, i2):
        self._fwd_columns(sh, i1, i2, ops=(1,))

    def _fwd_columns_own(self, sh, i1, i2):
        """only the rank's rows [r0, r0 + rcount) need to be right (MPFFT_SHARD_FWD_COLUMNS_OWN);
        the other rows are left as garbage, as the GPU stage leaves them unwritten"""
        self._fwd_columns(sh, i1, i2, rows=range(sh["r0"], sh["r0"] + sh["rcount"]))

    def _fwd_columns(self, sh, i1, i2, ops=(0, 1), rows=None):
        p = self.p
        mask = (1 << p.bits1) - 1
        ch = sh.get("src_chunk", 0)
        for k, op in ((0, i1), (1, i2)):
            if k not in ops:
                continue
            X = int.from_bytes(op.numpy().view(np.uint64).tobytes(), "little")
            for cl in range(sh["ccount"]):
                c = sh["c0"] + cl
                if ch:   # column slice: position jr's chunk starts at limb floor((jr NC + c0) bits1 / 64)
                    xs = [(X >> (64 * jr * ch + (jr * p.NC + c) * p.bits1 - 64 * p.slice_start(jr, sh["c0"] // p.C)))
                          & mask for jr in range(p.Tr)]
                else:
                    xs = [(X >> ((jr * p.NC + c) * p.bits1)) & mask for jr in range(p.Tr)]
                for pos in range(p.NR):
                    if rows is not None and pos not in rows:
                        self.put(sh["col"][k], self.col_slot(sh, pos, cl), 0x5A5A5A5A5A5A5A5A)   # garbage
                        continue
                    kr = revbin(pos, self.lbR)
                    v = sum(x * self.pw(p.w * p.NC * jr * kr) for jr, x in enumerate(xs) if x)
                    self.put(sh["col"][k], self.col_slot(sh, pos, cl), v)

    def stage_rows(self, name, sh, lo, hi):
        """a row stage on local rows [lo, hi) (the chunked row phase, GpuBackend.stage_rows)"""
        getattr(self, "_" + name)(sh, None, None, rows=range(lo, hi))

    def _fwd_rows(self, sh, i1, i2, rows=None):
        p = self.p
        for k in (0, 1):
            buf = sh["row"][k]
            for pl in (rows if rows is not None else range(sh["rcount"])):
                kr = revbin(sh["r0"] + pl, self.lbR)
                y = [self.get(buf, self.row_slot(sh, pl, c)) * self.pw(p.w * c * kr) for c in range(p.NC)]
                for q in range(p.NC):
                    kc = revbin(q, self.lbC)
                    self.put(buf, self.row_slot(sh, pl, q),
                             sum(y[c] * self.pw(p.w * p.NR * c * kc) for c in range(p.NC)))

    def _pointwise(self, sh, i1, i2, rows=None):
        A, B = sh["row"]
        for pl in (rows if rows is not None else range(sh["rcount"])):
            for c in range(self.p.NC):
                s = self.row_slot(sh, pl, c)
                self.put(A, s, self.get(A, s) * self.get(B, s))

    def _inv_rows(self, sh, i1, i2, rows=None):
        p = self.p
        buf = sh["row"][0]
        for pl in (rows if rows is not None else range(sh["rcount"])):
            kr = revbin(sh["r0"] + pl, self.lbR)
            x = [self.get(buf, self.row_slot(sh, pl, q)) for q in range(p.NC)]
            for c in range(p.NC):
                v = sum(x[q] * self.pw(-p.w * p.NR * c * revbin(q, self.lbC)) for q in range(p.NC))
                self.put(buf, self.row_slot(sh, pl, c), v * self.pw(-p.w * c * kr))

    def _inv_columns(self, sh, i1, i2):
        p = self.p
        buf = sh["col"][0]
        for cl in range(sh["ccount"]):
            x = [self.get(buf, self.col_slot(sh, pos, cl)) if pos < p.Tr else 0 for pos in range(p.NR)]
            self._itft(x, 0, p.NR, p.Tr)
            for jr in range(p.Tr):
                self.put(buf, self.col_slot(sh, jr, cl), x[jr] * self.pw(-(p.depth + 1)))

    # port of Exec::itft / itft1 / ifft_block / pairop (mpir-fft_amd/csrc/mpfft.hip)
    def _rho(self, m):
        p = self.p
        return p.w * p.NC * (p.NR // m)

    def _ifft_block(self, x, off, m):
        lb = log2(m)
        rho = self._rho(m)
        for lev in range(lb - 1, -1, -1):
            h = m >> (lev + 1)
            for pos in range(m):
                if pos & h:
                    continue
                e = (pos & (h - 1)) * (rho << lev)
                a, b = x[off + pos], x[off + pos + h] * self.pw(-e)
                x[off + pos], x[off + pos + h] = (a + b) % self.mod, (a - b) % self.mod

    def _pair(self, x, op, off, h, i0, cnt, rho):
        for i in range(i0, i0 + cnt):
            a, b = off + i, off + i + h
            e = i * rho
            if op == "double":
                x[a] = 2 * x[a] % self.mod
            elif op == "halfadd":
                x[a] = (x[a] + x[b]) * self.pw(-1) % self.mod
            elif op == "fill":
                x[b] = x[a] * self.pw(e) % self.mod
            elif op == "fix":
                d = x[a] - x[b]
                x[b] = d * self.pw(e) % self.mod
                x[a] = (x[a] + d) % self.mod
            elif op == "twoxmy":
                x[a] = (2 * x[a] - x[b]) % self.mod
            else:  # ibfly
                t = x[b] * self.pw(-e)
                x[a], x[b] = (x[a] + t) % self.mod, (x[a] - t) % self.mod

    def _itft(self, x, off, m, t):
        h = m // 2
        if t == m:
            return self._ifft_block(x, off, m)
        if t <= h:
            self._itft(x, off, h, t)
            return self._pair(x, "double", off, h, 0, t, 0)
        self._ifft_block(x, off, h)
        self._pair(x, "fill", off, h, t - h, h - (t - h), self._rho(m))
        self._itft1(x, off + h, h, t - h)
        self._pair(x, "ibfly", off, h, 0, t - h, self._rho(m))
        self._pair(x, "double", off, h, t - h, h - (t - h), 0)

    def _itft1(self, x, off, m, t):
        h = m // 2
        if t == m:
            return self._ifft_block(x, off, m)
        if t <= h:
            self._pair(x, "halfadd", off, h, t, h - t, 0)
            self._itft1(x, off, h, t)
            return self._pair(x, "twoxmy", off, h, 0, t, 0)
        self._ifft_block(x, off, h)
        self._pair(x, "fix", off, h, t - h, h - (t - h), self._rho(m))
        self._itft1(x, off + h, h, t - h)
        self._pair(x, "ibfly", off, h, 0, t - h, self._rho(m))

    # ---- combine (column layout, stripes) --------------------------------
    def halo_buffer(self):
        p = self.p
        return torch.zeros(p.Tr * p.H * p.l, dtype=torch.int64)

    def _coef(self, sh, j, kbase, k, halo):
        p = self.p
        if k < kbase:
            i = j * p.H + k - (kbase - p.H)
            limbs = halo[i * p.l:(i + 1) * p.l].numpy().view(np.uint64)
            return int.from_bytes(limbs.tobytes(), "little")
        assert k < kbase + p.C, "a stripe read past its own coefficients"
        return self.get(sh["col"][0], self.col_slot(sh, j, k - kbase))

    def combine(self, sh, phase, halo, sums_all=None):
        """same window-sum / carry semantics as k_combine1 / k_comb_summary / k_stripe_carry
        (combine.hpp): stripe j of rank g is product stripe j G + g"""
        p = self.p
        M64 = (1 << 64) - 1
        G, g = p.world, sh["c0"] // p.C
        if phase == 0:
            self._r = torch.zeros(p.Tr * p.SL, dtype=torch.int64)
            sums = []
            for j in range(p.Tr):
                s = j * G + g
                m0, m1, kbase = p.ms[s], p.ms[s + 1], s * p.C
                lo, hi = [], []
                for m in range(m0 - 1, m1):
                    if m < 0 or m1 == m0:
                        lo.append(0)
                        hi.append(0)
                        continue
                    P = 64 * m
                    klo = (P - p.N) // p.bits1 + 1 if P >= p.N else 0
                    khi = min((P + 63) // p.bits1, p.len - 1)
                    sw = 0
                    for k in range(klo, khi + 1):
                        st = k * p.bits1
                        cv = self._coef(sh, j, kbase, k, halo)
                        sw += ((cv << (st - P)) if st > P else (cv >> (P - st))) & M64
                    lo.append(sw & M64)
                    hi.append(sw >> 64)
                e = [lo[i + 1] + hi[i] for i in range(m1 - m0)]
                run, out = 0, []
                for v in e:
                    t = v + run
                    out.append(t & M64)
                    run = t >> 64
                if out:
                    arr = np.array(out, dtype=np.uint64).view(np.int64)
                    self._r[j * p.SL: j * p.SL + len(out)] = torch.from_numpy(arr.copy())
                sums += [run, 1 if all(v == M64 for v in e) else 0]
            return self._r, torch.tensor(sums, dtype=torch.int32)
        allv = torch.cat(list(sums_all)).tolist()
        for j in range(p.Tr):
            s = j * G + g
            cin = 0
            for q in range(s):   # stripes below s in product order ([rank][j] layout)
                e = (q % G) * p.Tr + q // G
                cin = 1 if (allv[2 * e] or (allv[2 * e + 1] and cin)) else 0
            if cin:
                n = p.ms[s + 1] - p.ms[s]
                v = int.from_bytes(self._r[j * p.SL: j * p.SL + n].numpy().view(np.uint64).tobytes(), "little") + 1
                v &= (1 << (64 * n)) - 1
                arr = np.frombuffer(v.to_bytes(8 * n, "little"), dtype=np.uint64).view(np.int64)
                self._r[j * p.SL: j * p.SL + n] = torch.from_numpy(arr.copy())
        return self._r
