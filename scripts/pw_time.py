#!/usr/bin/env python3
"""Time the pointwise stage alone (mpfft_stage POINTWISE) on a C3- or C4-shaped workspace
filled with random reduced-form coefficients; prints ms per launch.  Timing only (the
inputs are arbitrary residues).  usage: pw_time.py [C3|C4] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import mpfft_loader  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
depth, w, nl = {"C3": (15, 4, 20312500), "C4": (17, 2, 156250000), "C2": (15, 4, 15625000)}[cfg]
mp = mpfft_loader.load()
dev = torch.device("cuda:0")
P = mp.plan_info(nl, nl, depth, w)
lay = mp.workspace_layout(nl, nl, depth, w)
ws = mp.alloc_workspace(nl, nl, depth, w, dev)
g = torch.Generator(device=dev)
g.manual_seed(1)
u8 = ws.view(torch.uint8)
T, l = P["trunc"], P["l"]
for k in ("digA", "digB"):
    v = u8[lay[k]: lay[k] + T * l * 8].view(torch.int64)
    v.random_(generator=g)
for k in ("topA", "topB"):
    u8[lay[k]: lay[k] + T * 4].zero_()
for k in ("cbA", "cbB"):
    u8[lay[k]: lay[k] + T * lay["cbw"] * 8].zero_()
da = torch.zeros(1, dtype=torch.int64, device=dev)
dr = torch.zeros(1, dtype=torch.int64, device=dev)
kern = mp.stage_kernels(nl, nl, depth, w)["pointwise"]
for _ in range(2):
    mp.stage(mp.STAGE_POINTWISE, da, da, dr, nl, nl, depth, w, ws)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    mp.stage(mp.STAGE_POINTWISE, da, da, dr, nl, nl, depth, w, ws)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"{cfg} pointwise {kern}: {ms:.3f} ms per launch ({T} slots, {ms * 1e6 / T:.1f} ns/slot) "
      f"variant={os.environ.get('MPFFT_PW_VARIANT', '-')}")
