"""Diagnostics (GPU box): forward-stage values of one shape with some k_rpass modes
switched off (MPFFT_RPASS_OFF), compared slot by slot mod p with an exact reference
(gpu_stages spec).  Needs the diagnostic build (make -C mpir-fft_amd/csrc DIAG=1) and
MPFFT_LIB=diag.  usage: MPFFT_LIB=diag python scripts/dbg_rpass.py depth w n1 n2 [stage]"""
import os
import sys

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from helpers import chunks, log2, revbin, to_int  # noqa: E402
from gpu_stages import _t, _slots, _cbs, _val_reduced  # noqa: E402


def main():
    import torch
    import mpfft_loader
    mp = mpfft_loader.load()
    depth, w, n1, n2 = map(int, sys.argv[1:5])
    upto = sys.argv[5] if len(sys.argv) > 5 else "cols"
    a = mp.fill_random(n1, 1000 + depth * 7 + n1)
    b = mp.fill_random(n2, 2000 + w * 3 + n2)
    P = mp.plan_info(n1, n2, depth, w)
    n, l, NC, NR, T, bits1 = P["n"], P["l"], P["NC"], P["NR"], P["trunc"], P["bits1"]
    N = n * w
    p = (1 << N) + 1
    Tr = T // NC
    lbR, lbC = log2(NR), log2(NC)
    xa = chunks(to_int(a), 2 * n, bits1)
    dev = torch.device("cuda:0")
    da, db = _t(a, dev), _t(b, dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace(n1, n2, depth, w, dev)
    ws.fill_(0x5A if os.environ.get('POISON', '1') == '1' else 0)
    mp.stage(mp.STAGE_FWD_COLUMNS, da, db, dr, n1, n2, depth, w, ws)
    if upto == "rows":
        mp.stage(mp.STAGE_FWD_ROWS, da, db, dr, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    dig, top = _slots(mp, ws, n1, n2, depth, w, 0)
    cb = _cbs(mp, ws, n1, n2, depth, w, 0)

    def X(x, k):
        acc = 0
        for j, xj in enumerate(x):
            if xj:
                e = (w * j * k) % (2 * N)
                acc += xj << e if e < N else -(xj << (e - N))
        return acc % p
    bad = []
    for pp in range(Tr):
        for q in range(NC):
            s = pp * NC + q
            if upto == "rows":
                k = revbin(pp, lbR) + NR * revbin(q, lbC)
                want = X(xa, k)
            else:
                # column DIF output at position pp of column q: sum_r x_(r NC + q) w^(r revbin(pp)) (mod p),
                # w = 2^(w NC), times the MFA twiddle? no: columns before twiddle
                want = sum(xa[r * NC + q] << 0 for r in range(0)) if False else None
                col = [xa[r * NC + q] for r in range(NR)]
                kk = revbin(pp, lbR)
                acc = 0
                for r, xr in enumerate(col):
                    if xr:
                        e = (w * NC * r * kk) % (2 * N)
                        acc += xr << e if e < N else -(xr << (e - N))
                want = acc % p
            got = _val_reduced(dig, top, cb, s, N) % p
            if got != want:
                bad.append((pp, q, int(top[s])))
                if len(bad) <= 3:
                    d = (got - want) % p
                    dn = (want - got) % p
                    for name, v in (("got-want", d), ("want-got", dn)):
                        bits = [i for i in range(N + 1) if (v >> i) & 1]
                        print(name, "popcount", len(bits), "lowest bits", bits[:6], "bitlen", v.bit_length())
    print("OFF=%s POISON=%s %s: %d bad of %d" % (os.environ.get("MPFFT_RPASS_OFF", "0"), os.environ.get("POISON", "1"), upto, len(bad), Tr * NC), bad[:12] if os.environ.get("ALL") is None else bad)


if __name__ == "__main__":
    main()
