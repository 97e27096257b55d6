#!/usr/bin/env python3
"""GPU sweep for the (depth, w) chooser (mpfft_choose, csrc/mpfft.hip): for every
coefficient size l = 2^k limbs (k = 0..12) one large configuration is timed (device-
resident multiplies, HBM operands) and the per-slot cost is recorded.  Output:
profiles/r02/chooser_sweep.json; the table in mpfft.hip (CHOOSE_SLOT_NS) is copied
from it.  usage: python scripts/chooser_sweep.py [out.json]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import mpfft_loader
    from helpers import max_limbs
    mp = mpfft_loader.load()
    dev = torch.device("cuda:0")
    rows = []
    for k in range(13):
        d = min(25 - k, k + 6)
        w = (64 << k) >> d
        n = max_limbs(d, w)
        P = mp.plan_info(n, n, d, w)
        a = torch.from_numpy(mp.fill_random(n, 11).view(np.int64)).to(dev)
        b = torch.from_numpy(mp.fill_random(n, 12).view(np.int64)).to(dev)
        r = torch.zeros(2 * n, dtype=torch.int64, device=dev)
        ws = mp.alloc_workspace(n, n, d, w, dev)
        mp.mul_device(r, a, n, b, n, d, w, ws)
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            mp.mul_device(r, a, n, b, n, d, w, ws)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        rows.append({"k": k, "l": 1 << k, "depth": d, "w": w, "n": n, "trunc": P["trunc"], "ms": ms,
                     "ns_per_slot": ms * 1e6 / P["trunc"]})
        print(json.dumps(rows[-1]), flush=True)
        del a, b, r, ws
        torch.cuda.empty_cache()
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "chooser_sweep.json")
    json.dump(rows, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
