"""Stage-by-stage GPU checks against exact big-integer math (used by
tests/test_gpu_parity.py; runnable directly on the GPU box for diagnostics:
`python tests/gpu_stages.py`).

Stage specs:
  forward  slot p*NC + q = X_{revbin(p) + NR revbin(q)} mod 2^N + 1 (canonical, or
           reduced when the pointwise is k_pwss),
           X_k = sum_j x_j 2^(w j k) (a3 output spec, up to the reference's two
           revbin permutations which this build never performs), p < T/NC
  pointwise slot = XA * XB mod 2^N + 1, reduced form (limbs + carry masks) (a20)
  inverse  slot j = c_j = sum_i a_i b_(j-i), exact, j < trunc           (a13, a21)
  combine  r = i1 * i2                                                  (a22)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from helpers import chunks, log2, revbin, to_int  # noqa: E402


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def _slots(mp, ws, n1, n2, depth, w, which):
    digA, topA, digB, topB = mp.workspace_views(ws, n1, n2, depth, w)
    dig, top = (digA, topA) if which == 0 else (digB, topB)
    return dig.cpu().numpy().view(np.uint64), top.cpu().numpy().astype(np.int64)


def _cbs(mp, ws, n1, n2, depth, w, which):
    """carry masks of the reduced form: word 2W (2W+1) bit k = limb 64W+k carries +1 (-1)"""
    lay = mp.workspace_layout(n1, n2, depth, w)
    off, cbw, slots = lay["cbA" if which == 0 else "cbB"], lay["cbw"], lay["slots"]
    u8 = ws.view(__import__("torch").uint8)
    return u8[off:off + slots * cbw * 8].view(__import__("torch").int64).view(slots, cbw).cpu().numpy().view(np.uint64)


def _val(dig, top, s, N):
    return to_int(dig[s]) + int(top[s]) * (1 << N)


def _val_reduced(dig, top, cb, s, N):
    """value of a reduced-form slot: limbs + carries (limb m's carry lands at 2^(64(m+1)),
    limb l-1's at 2^N) + top 2^N"""
    v = _val(dig, top, s, N)
    for W in range(len(cb[s]) // 2):
        pos, neg = int(cb[s][2 * W]), int(cb[s][2 * W + 1])
        for k in range(64):
            if (pos >> k) & 1:
                v += 1 << (64 * (64 * W + k + 1))
            if (neg >> k) & 1:
                v -= 1 << (64 * (64 * W + k + 1))
    return v


def _canonical(dig, top, s):
    t = int(top[s])
    return t == 0 or (t == 1 and not dig[s].any())


def _convolution(ca, cb, N, T, mul=None):
    """c_j = sum_i ca_i cb_(j-i) for j < T (each c_j < 2^(N+1)): one Kronecker product with
    (N + 64)-bit slots; `mul` multiplies limb arrays (GMP mpn_mul via the oracle) when given."""
    S = N + 64
    def pack(c):
        return b"".join(v.to_bytes(S // 8, "little") for v in c)
    if mul is None:
        C = int.from_bytes(pack(ca), "little") * int.from_bytes(pack(cb), "little")
    else:
        r = mul(np.frombuffer(pack(ca), dtype=np.uint64), np.frombuffer(pack(cb), dtype=np.uint64))
        C = int.from_bytes(np.ascontiguousarray(r).tobytes(), "little")
    mask = (1 << S) - 1
    return [(C >> (j * S)) & mask for j in range(T)]


def run_stages(mp, depth, w, a, b, dev="cuda:0", check=("fwd", "pw", "inv", "comb"), mul=None):
    """Returns a list of failure strings (empty = all stages exact)."""
    import torch
    n1, n2 = len(a), len(b)
    P = mp.plan_info(n1, n2, depth, w)
    n, l, NC, NR, T, bits1 = P["n"], P["l"], P["NC"], P["NR"], P["trunc"], P["bits1"]
    N = n * w
    p = (1 << N) + 1
    Tr = T // NC
    lbR, lbC = log2(NR), log2(NC)
    A, B = to_int(a), to_int(b)
    xa = chunks(A, 2 * n, bits1)
    xb = chunks(B, 2 * n, bits1)
    dev = torch.device(dev)
    da, db = _t(a, dev), _t(b, dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace(n1, n2, depth, w, dev)
    ws.fill_(0x5A)   # poison: nothing may read slots it did not write
    fails = []

    def X(x, k):
        # sum_j x_j 2^(w j k) mod p, with 2^e == -2^(e - N) for N <= e < 2N (shifts, no modexp)
        acc = 0
        for j, xj in enumerate(x):
            if xj:
                e = (w * j * k) % (2 * N)
                acc += xj << e if e < N else -(xj << (e - N))
        return acc % p

    mp.stage(mp.STAGE_FWD_COLUMNS, da, db, dr, n1, n2, depth, w, ws)
    mp.stage(mp.STAGE_FWD_ROWS, da, db, dr, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    XA, XB = {}, {}
    for which, x, store in ((0, xa, XA), (1, xb, XB)):
        dig, top = _slots(mp, ws, n1, n2, depth, w, which)
        cbx = _cbs(mp, ws, n1, n2, depth, w, which)
        for pp in range(Tr):
            for q in range(NC):
                s = pp * NC + q
                k = revbin(pp, lbR) + NR * revbin(q, lbC)
                want = X(x, k)
                store[s] = want
                if "fwd" in check:
                    # canonical, or (k_pwss loads it) the reduced form: limbs + carries + top, mod p
                    got = _val_reduced(dig, top, cbx, s, N) % p
                    if got != want:
                        fails.append(f"fwd op{which} slot ({pp},{q}) k={k}: got {got:x} top {top[s]} want {want:x}")
                        if len(fails) > 8:
                            return fails
    mp.stage(mp.STAGE_POINTWISE, da, db, dr, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    if "pw" in check:
        dig, top = _slots(mp, ws, n1, n2, depth, w, 0)
        cbA = _cbs(mp, ws, n1, n2, depth, w, 0)
        for s in range(T):
            want = XA[s] * XB[s] % p
            got = _val_reduced(dig, top, cbA, s, N) % p    # reduced form (what the inverse pass loads)
            if got != want:
                fails.append(f"pointwise slot {s}: got {got:x} (top {top[s]}) want {want:x}")
                if len(fails) > 8:
                    return fails
    for st in (mp.STAGE_INV_ROWS, mp.STAGE_INV_COLUMNS, mp.STAGE_SCALE):
        mp.stage(st, da, db, dr, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    if "inv" in check:
        dig, top = _slots(mp, ws, n1, n2, depth, w, 0)
        ca = chunks(A, P["j1"], bits1)
        cb = chunks(B, P["j2"], bits1)
        cw = _convolution(ca, cb, N, T, mul)
        for j in range(T):
            want = cw[j]
            got = _val(dig, top, j, N)
            if got != want:
                fails.append(f"inverse coeff {j}: got {got:x} (top {top[j]}) want {want:x}")
                if len(fails) > 8:
                    return fails
    mp.stage(mp.STAGE_COMBINE, da, db, dr, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    if "comb" in check:
        got = to_int(dr.cpu().numpy().view(np.uint64))
        if got != A * B:
            fails.append("combine: product differs")
    return fails


if __name__ == "__main__":
    import mpfft_loader
    mp = mpfft_loader.load()
    shapes = [(6, 1, 3, 2), (6, 1, 1, 1), (7, 1, 5, 4), (8, 2, 30, 25), (8, 4, 60, 50), (9, 1, 30, 31), (10, 3, 300, 200)]
    for depth, w, n1, n2 in shapes:
        a = mp.fill_random(n1, 1000 + depth)
        b = mp.fill_random(n2, 2000 + w)
        f = run_stages(mp, depth, w, a, b)
        print(depth, w, n1, n2, "OK" if not f else "FAIL")
        for line in f[:6]:
            print("   ", line[:300])
