#!/usr/bin/env python3
"""A/B of the MFA split at l = 2048 (make_plan, csrc/mpfft.hip): times device-resident
multiplies over a range of truncation ratios T / 2n with the diagnostic library's
MPFFT_SPLIT=ref|alt (set in the environment; one process per setting, the knob is read once).
usage: MPFFT_LIB=diag MPFFT_SPLIT=alt python scripts/split_sweep.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(15, 4, r) for r in (0.40, 0.48, 0.52, 0.58, 0.65, 0.75, 0.85, 0.95)] + \
         [(14, 8, r) for r in (0.45, 0.55, 0.8)] + [(16, 2, r) for r in (0.45, 0.6, 0.9)] + [(13, 16, 0.7)]


def main():
    import torch
    import mpfft_loader
    mp = mpfft_loader.load()
    dev = torch.device("cuda:0")
    for d, w, r in SHAPES:
        n = int(r * (1 << d) * 1024)
        P = mp.plan_info(n, n, d, w)
        a = torch.from_numpy(mp.fill_random(n, 11).view(np.int64)).to(dev)
        b = torch.from_numpy(mp.fill_random(n, 12).view(np.int64)).to(dev)
        res = torch.zeros(2 * n, dtype=torch.int64, device=dev)
        ws = mp.alloc_workspace(n, n, d, w, dev)
        mp.mul_device(res, a, n, b, n, d, w, ws)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(3):
                mp.mul_device(res, a, n, b, n, d, w, ws)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 3 * 1e3)
        print(json.dumps({"split": os.environ.get("MPFFT_SPLIT", "default"), "depth": d, "w": w, "n": n,
                          "ratio": round(P["trunc"] / (2 * P["n"]), 3), "NC": P["NC"], "NR": P["NR"],
                          "ms": round(best, 3)}), flush=True)
        del a, b, res, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
