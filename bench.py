#!/usr/bin/env python3
"""Benchmark: limbs/s of new_mpn_mul on MI355X (BASELINE.json metric).

A "step" is one full new_mpn_mul (split -> forward truncated MFA of both
operands -> pointwise mulmod -> inverse MFA -> scale -> combine) of two
synthetic operands already resident in HBM.  Default workload = BASELINE.json
configs[1] (C1: depth 11, w 8, l = 256 limbs per coefficient, two 261952-limb
operands).  value = (n1 + n2) * steps * world / max-rank time.

Multi-GPU (`--gpus N` under torch.distributed.run): every rank multiplies its
own operand pair (independent products, no data-path collective; scaling
"weak").  The column-sharded single-product path with the RCCL all-to-all is
`--mode sharded` (see mpir-fft_amd/sharded.py).

Extra fields: "roofline" for the dominant kernel (time from HIP events on the
library's stream inside the timed region), "stages" (per-stage ms), and
"cpu_baseline": the oracle (oracle/, a CPU restatement of the reference,
kind "port") timed on this host, rank 0 at N = 1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "limbs/s for new_mpn_mul N×N-bit at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)

# (depth, w, limbs per operand) -- SURVEY Appendix C / BASELINE.md
CONFIGS = {
    "C0": (11, 1, 16384),
    "C1": (11, 8, 261952),
    "C2": (15, 4, 15625000),
    "C3": (15, 4, 20312500),
    "C4": (17, 2, 156250000),
}
SEED1, SEED2 = 0x1001, 0x2002

STAGE_NAMES = ["fwd_columns", "fwd_rows", "pointwise", "inv_rows", "inv_columns", "scale", "combine"]
STAGE_KERNEL = {"pointwise": "k_pwm (negacyclic products on v_mfma_i32_32x32x32_i8)", "scale": "k_scale",
                "combine": "k_comb_sum + k_carry_*"}
I8_MFMA_PEAK = 5.0e15      # int8 ops/s dense: 2x the 2.5 PF BF16 rate per clock (MI355X_MICROARCH.md)


def pointwise_ops(P):
    """Algorithmic int8 ops of one pointwise launch: T products of two 8l-byte numbers,
    (8l)^2 byte MACs each, 2 ops per MAC (the schoolbook the int8 MFMA path executes)."""
    return P["trunc"] * 2 * (8 * P["l"]) ** 2


def stage_bytes(P, name, n1, n2):
    """Algorithmic HBM bytes of one launch of a stage (DESIGN.md "Roofline accounting")."""
    T, l = P["trunc"], P["l"]
    blk = 8 * l + 4                         # one coefficient: l limbs + carry limb
    if name == "fwd_columns":               # read operands, write 2 * T blocks
        return 8 * (n1 + n2) + 2 * T * blk
    if name in ("fwd_rows",):
        return 2 * 2 * T * blk
    if name == "pointwise":                 # read A, B, write A
        return 3 * T * blk
    if name in ("inv_rows", "inv_columns", "scale"):
        return 2 * T * blk
    if name == "combine":                   # read T blocks, write the product
        return T * blk + 8 * (n1 + n2)
    raise KeyError(name)


def b_alg(P, n1, n2):
    """minimum traffic of the three-pass MFA, 8A + 16 (n1 + n2)."""
    A = P["trunc"] * (P["l"] + 1) * 8
    return 8 * A + 16 * (n1 + n2)


def cpu_baseline(a, b, depth, w, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    reps, t0 = 0, time.perf_counter()
    ref = None
    while True:
        ref = O.new_mpn_mul(a, b, depth, w)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 1000:
            break
    return {"value": (len(a) + len(b)) * reps / el, "unit": "limbs/s", "cores": 1, "kind": "port",
            "sample": f"{reps} full new_mpn_mul of the same operands via oracle/ (single thread), {el:.1f} s"}, ref


def pmc_traffic(cfg):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc summary, if any."""
    p = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C1", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="replicas", choices=["replicas", "sharded"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import mpfft_loader
    mp = mpfft_loader.load()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.mode == "sharded":
        from importlib import import_module
        sh = import_module("mpir_fft_amd.sharded")
        res = sh.bench(args, CONFIGS[args.config], rank, world, dev)
        if rank == 0:
            print(json.dumps(res))
        if world > 1:
            dist.destroy_process_group()
        return

    depth, w, nl = CONFIGS[args.config]
    n1 = n2 = nl
    P = mp.plan_info(n1, n2, depth, w)
    a = mp.fill_random(n1, SEED1 + 0x10000 * rank)
    b = mp.fill_random(n2, SEED2 + 0x10000 * rank)
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace(n1, n2, depth, w, dev)
    stream = torch.cuda.Stream(device=dev)

    def step_full():
        mp.mul_device(dr, da, n1, db, n2, depth, w, ws, stream=stream)

    def step(events=None):
        for si, _ in enumerate(STAGE_NAMES):
            if events is not None:
                events[si].record(stream)
            mp.stage(si, da, db, dr, n1, n2, depth, w, ws, stream=stream)
        if events is not None:
            events[len(STAGE_NAMES)].record(stream)

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step_full()
    torch.cuda.synchronize(dev)

    # timed region: K whole multiplies, one library call each (no per-stage events:
    # an event record between two kernels costs ~5 us of idle GPU)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step_full()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # stage breakdown: the same K multiplies again, stage by stage, with HIP events
    # recorded on the library's stream around every stage
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(STAGE_NAMES) + 1)] for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    for k in range(args.steps):
        step(ev[k])
    torch.cuda.synchronize(dev)
    stage_ms = np.zeros(len(STAGE_NAMES))
    for k in range(args.steps):
        for si in range(len(STAGE_NAMES)):
            stage_ms[si] += ev[k][si].elapsed_time(ev[k][si + 1])
    stage_ms /= args.steps

    exact = None
    if not args.no_check and rank == 0:
        got = dr.cpu().numpy().view(np.uint64)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        exact = bool((got == O.gmp_mul(a, b)).all())

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_step = el / args.steps * 1e3
    value = world * (n1 + n2) * args.steps / el
    dom = int(np.argmax(stage_ms))
    dname = STAGE_NAMES[dom]
    dbytes = stage_bytes(P, dname, n1, n2)
    achieved = dbytes / (stage_ms[dom] * 1e-3)
    if dname == "pointwise" and P["l"] % 128 == 0:     # matrix-core kernel: priced against the int8 MFMA peak
        ops = pointwise_ops(P)
        roof = {"bound": "mfma", "achieved": ops / (stage_ms[dom] * 1e-3) / 1e12, "peak": I8_MFMA_PEAK / 1e12,
                "unit": "TFLOP/s", "op_type": "int8 MAC ops (2 per MAC), TOP/s",
                "frac": ops / (stage_ms[dom] * 1e-3) / I8_MFMA_PEAK, "alg_ops_per_launch": ops,
                "hbm_achieved_GBps": achieved / 1e9, "alg_bytes_per_launch": dbytes}
    else:
        roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "alg_bytes_per_launch": dbytes}
    pmc = pmc_traffic(args.config)
    traffic = None
    if pmc and pmc.get("stage") == dname:
        traffic = pmc.get("hbm_bytes_per_launch")
    balg = b_alg(P, n1, n2)
    dev_ms = float(stage_ms.sum())
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "limbs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (xoshiro256** limbs, seeds 0x1001/0x2002 per rank)",
        "config": {"workload": f"{args.config}: new_mpn_mul depth={depth} w={w} n1=n2={nl} limbs "
                               f"(l={P['l']} limbs/coeff, NC x NR = {P['NC']} x {P['NR']}, trunc={P['trunc']})",
                   "parallelism": f"replicas x{world}" if world > 1 else "single"},
        "roofline": dict(roof, kernel=STAGE_KERNEL.get(dname, "k_lpass (" + dname + ")"), stage=dname,
                         traffic=traffic, avg_ms=float(stage_ms[dom])),
        "pipeline": {"device_ms": dev_ms, "b_alg_bytes": balg,
                     "hbm_frac_b_alg": balg / (dev_ms * 1e-3) / HBM_PEAK},
        "stages_ms": {n: float(t) for n, t in zip(STAGE_NAMES, stage_ms)},
        "stage_timing": "separate K-multiply pass after the timed region, HIP events per stage on the library stream",
        "exact": exact,
    }
    if world == 1 and not args.no_cpu_baseline:
        cb, ref = cpu_baseline(a, b, depth, w, args.cpu_budget)
        res["cpu_baseline"] = cb
        res["exact_vs_port"] = bool((dr.cpu().numpy().view(np.uint64) == ref).all())
    print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
