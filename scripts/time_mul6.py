#!/usr/bin/env python3
"""MI355X timing of the sqrt2 front end new_mpn_mul6 (mul_fft.c:3573) next to new_mpn_mul
(:3190) on the same operands: device-resident multiplies timed with HIP events around K
calls on one stream.  Shapes: (depth, w) for mul6 and the new_mpn_mul pair with the same
coefficient size and transform length (mul6 at depth d, w == new_mpn_mul at depth d+1, w/2
for even w).  usage: python scripts/time_mul6.py [out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps, torch, stream):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import torch
    import mpfft_loader
    mp = mpfft_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    rows = []
    # (mul6 depth, w, n limbs, new_mpn_mul depth, w)
    cases = [(14, 8, 20312500, 15, 4),        # C3-size operands, l = 2048
             (10, 16, 261952, 11, 8),         # C1-size operands, l = 256
             (14, 1, 3142656, None, None),    # test_mul4's shape (odd w: sqrt2 twiddles), l = 256
             (15, 1, 8388352, None, None)]    # odd w, l = 512
    for d6, w6, n, d, w in cases:
        a = mp.fill_random(n, 0x1001)
        b = mp.fill_random(n, 0x2002)
        da = torch.from_numpy(a.view(np.int64)).to(dev)
        db = torch.from_numpy(b.view(np.int64)).to(dev)
        dr = torch.zeros(2 * n, dtype=torch.int64, device=dev)
        row = {"n1": n, "n2": n, "mul6": {"depth": d6, "w": w6, **mp.plan_info6(n, n, d6, w6)}}
        ws = mp.alloc_workspace6(n, n, d6, w6, dev)
        with torch.cuda.stream(stream):
            ms6 = timed(lambda: mp.mul6_device(dr, da, n, db, n, d6, w6, ws, stream=stream), 5, torch, stream)
        r6 = dr.cpu().numpy().view(np.uint64).copy()
        row["mul6"]["ms"] = ms6
        row["mul6"]["limbs_per_s"] = 2 * n / (ms6 * 1e-3)
        del ws
        if d is not None:
            ws = mp.alloc_workspace(n, n, d, w, dev)
            with torch.cuda.stream(stream):
                ms = timed(lambda: mp.mul_device(dr, da, n, db, n, d, w, ws, stream=stream), 5, torch, stream)
            r = dr.cpu().numpy().view(np.uint64)
            row["mul"] = {"depth": d, "w": w, "ms": ms, "limbs_per_s": 2 * n / (ms * 1e-3),
                          "same_product": bool((r == r6).all())}
            del ws
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
