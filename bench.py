#!/usr/bin/env python3
"""Benchmark: limbs/s of new_mpn_mul on MI355X (BASELINE.json metric).

A "step" is one full new_mpn_mul (split -> forward truncated MFA of both
operands -> pointwise mulmod -> inverse MFA -> scale -> combine) of two
synthetic operands already resident in HBM.  value = (n1 + n2) * steps / time.

Workloads:
  N = 1 (default): C3 -- 1.3e9-bit x 1.3e9-bit, depth 15, w 4, l = 2048 limbs per
         coefficient, odd truncation point (BASELINE configs[3], the largest single-GPU
         config); --config selects C0..C4 (C4 = 1e10 bits fits one MI355X too).
  N > 1: C4 -- 1e10-bit operands, MFA columns sharded over the N ranks with RCCL
         all-to-alls between the column and row passes (BASELINE configs[4],
         mpir-fft_amd/sharded.py); "strong" scaling (one product split N ways).
         `python bench.py --gpus N` with no torch.distributed environment launches
         the N rank processes itself (torch.distributed.run, before any GPU call).

Fields beyond the driver contract:
  roofline      the dominant kernel (largest stage time): algorithmic HBM bytes per
                launch / its average duration from HIP events recorded inside the
                timed region on the library's stream; traffic = FETCH+WRITE bytes per
                launch from profiles/pmc_<config>.json (rocprofv3 --pmc, corrected as
                MI355X_MICROARCH.md prescribes) when present.
  pipeline      whole multiply vs the HBM roofline: B_alg = 8A + 16(n1+n2).
  e2e_host      host-pointer new_mpn_mul (H2D + multiply + D2H), the drop-in boundary.
  cpu_baseline  oracle/ (CPU restatement of the reference, kind "port", 1 thread) on
                the same operands, plus GMP mpn_mul, CPU model and nproc (rank 0, N = 1).
"""
import argparse
import hashlib
import json
import statistics
import os
import socket
import subprocess
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
# --mul6: the sqrt2 front end new_mpn_mul6 (mul_fft.c:3573) -- (depth, w, limbs): C3's operands
# through a length-4n transform of the same coefficient size, and test_mul4's shape (:5559)
CONFIGS6 = {
    "C3": (14, 8, 20312500),
    "M4": (14, 1, 3142656),
}


def stage_bytes(P, name, n1, n2):
    """Algorithmic HBM bytes of one multiply's stage (every launch of it together)."""
    T, l = P["trunc"], P["l"]
    blk = 8 * l + 4                         # one coefficient: l limbs + carry limb
    if name == "fwd_columns":               # read operands, write 2 T blocks
        return 8 * (n1 + n2) + 2 * T * blk
    if name == "fwd_rows":                  # both operands in and out
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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(a, b, depth, w, reps, warmup=1):
    """oracle/ new_mpn_mul (1 thread) on the bench operands, pinned to one core (BASELINE.md's
    `taskset -c 0` protocol): `warmup` untimed calls, then the median of `reps` timed calls;
    GMP mpn_mul on the same operands beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        ref = None
        for _ in range(warmup):
            ref = O.new_mpn_mul(a, b, depth, w)
        times = []
        for _ in range(max(1, reps)):
            t0 = time.perf_counter()
            ref = O.new_mpn_mul(a, b, depth, w)
            times.append(time.perf_counter() - t0)
        t1 = time.perf_counter()
        g = O.gmp_mul(a, b)
        tg = time.perf_counter() - t1
    finally:
        os.sched_setaffinity(0, old)
    med = statistics.median(times)
    n = len(a) + len(b)
    return {"value": n / med, "unit": "limbs/s", "cores": 1, "kind": "port",
            "sample": f"median of {len(times)} full new_mpn_mul calls of the bench operands via oracle/ "
                      f"(CPU restatement of mul_fft.c:3190, single thread pinned to core {core}) after "
                      f"{warmup} warm-up: {med:.2f} s per call (min {min(times):.2f}, max {max(times):.2f})",
            "seconds_per_call": times,
            "gmp_mpn_mul_limbs_per_s": n / tg, "gmp_mpn_mul_s": tg,
            "cpu_model": cpu_model(), "nproc": os.cpu_count()}, ref, g


def cpu_ncore(cfg, procs):
    """The host's multi-core capacity beside the 1-core contract number (VERDICT r5 #6,
    BASELINE.md's optional nproc-way figure): oracle/ncore.py runs K = min(procs, allowed cores,
    free RAM / 4 GB) concurrent independent CPU new_mpn_mul calls of the bench operands, one
    process per core, then K concurrent GMP mpn_mul calls.  Run before this process touches the
    GPU; the workers import no torch."""
    depth, w, nl = CONFIGS[cfg]
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "ncore.py"), "--procs", str(procs), "--depth", str(depth),
           "--w", str(w), "--n", str(nl), "--seed1", str(SEED1), "--seed2", str(SEED2)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    except Exception as e:   # reported, never fatal: the 1-core figure is the contract number
        return {"error": repr(e)}


VALU_PEAK = 1024 * 32 * 2.4e9   # int32 lane-ops/s: 256 CUs x 4 SIMD-32 x 2.4 GHz (MI355X_MICROARCH.md)


def pmc_record(cfg, kernel):
    """The committed rocprofv3 --pmc record of `kernel` for this config (profiles/pmc_<cfg>.json,
    built by scripts/pmc_merge.py): HBM bytes per launch and the SQ limiter counters."""
    p = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    want = kernel.split(" ")[0]                    # e.g. "k_pwss<20>" -> matches "void k_pwss<20, 8, 1>(...)"
    stem, tmpl = want.split("<")[0], want[len(want.split("<")[0]):].strip("<>")
    for name, rec in d.get("kernels", {}).items():
        base = name.replace("void ", "").split("(")[0]
        if base.split("<")[0] == stem and (not tmpl or base.split("<", 1)[-1].startswith(tmpl)):
            return rec, os.path.relpath(p, ROOT)
    return None, None


def roofline(cfg, kernel, stage, alg_bytes, avg_ms):
    """Roofline of the dominant kernel against HBM: its algorithmic bytes per launch
    over its live average duration, vs 8 TB/s -- the headline `frac`.  The kernel's actual
    limiter is reported beside it, not in its place: the VALU issue rate of its executed
    instructions (SQ_INSTS_VALU per launch from the committed counter pass x 64 lanes / the
    live duration, against 1024 SIMD-32 x 2.4 GHz; it credits overhead instructions too, so it
    is a limiter, not algorithmic work) and the other SQ counters of the same pass."""
    sec = avg_ms * 1e-3
    hbm = {"achieved": alg_bytes / sec / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
           "frac": alg_bytes / sec / HBM_PEAK}
    rec, src = pmc_record(cfg, kernel)
    traffic = rec.get("hbm_bytes_per_launch") if rec else None
    out = {"bound": "hbm", **hbm, "traffic": traffic, "traffic_source": src, "kernel": kernel, "stage": stage,
           "avg_ms": avg_ms, "alg_bytes_per_launch": alg_bytes,
           "timing": "HIP events on the library stream at the stage boundaries of K profiled multiplies "
                     "(a separate loop after the timed one)"}
    if rec and rec.get("SQ_INSTS_VALU"):
        valu = rec["SQ_INSTS_VALU"] * 64 / sec
        lim = {k: rec[k] for k in ("valu_issue_util", "valu_cycle_util_est", "lds_util", "wait_inst_frac",
                                   "wait_any_frac", "waves_per_simd", "clock_ghz") if k in rec}
        lim.update({"valu_achieved_TOPs": valu / 1e12, "valu_peak_TOPs": VALU_PEAK / 1e12,
                    "valu_frac": valu / VALU_PEAK, "valu_insts_per_launch": rec["SQ_INSTS_VALU"],
                    "source": src,
                    "note": "executed int32 VALU lane-ops / the live duration vs 1024 SIMD-32 x 2.4 GHz: "
                            "the limiter of a latency/VALU-bound kernel (HBM frac is the roofline axis)"})
        out["limiters"] = lim
    return out


def single_gpu_line(mp, dev, cfg, steps, warmup, check=True):
    """One-GPU device-resident multiplies of `cfg` (the single-GPU path), timed like the headline
    line: the N = 1 point of the sharded C4 curve (bench.py --gpus N splits the same product)."""
    import torch
    depth, w, nl = CONFIGS[cfg]
    a = mp.fill_random(nl, SEED1)
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    del a
    b = mp.fill_random(nl, SEED2)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    del b
    dr = torch.zeros(2 * nl, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace(nl, nl, depth, w, dev)
    stream = torch.cuda.Stream(device=dev)
    for _ in range(warmup):
        mp.mul_device(dr, da, nl, db, nl, depth, w, ws, stream=stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        mp.mul_device(dr, da, nl, db, nl, depth, w, ws, stream=stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    exact = None
    if check:
        want = golden_digest(cfg)
        exact = hashlib.sha256(dr.cpu().numpy().tobytes()).hexdigest() == want if want else None
    del da, db, dr, ws
    torch.cuda.empty_cache()
    return {"config": cfg, "path": "single GPU (mpfft_mul_device)", "n_gpus": 1, "steps": steps,
            "ms_per_step": el / steps * 1e3, "value": 2 * nl * steps / el, "unit": "limbs/s", "exact": exact}


def multi_entry_line(mp, cfg, devices, steps, warmup, check=True, host_reps=1):
    """The one-process C entry over `devices` (rank g on devices[g]; a device may repeat -- the
    one-GPU rehearsal), as a sub-record: mpfft_mul_multi_device on packed operand slices already
    resident on the devices (device time: K calls ordered on per-rank streams, all devices
    synchronised around them), the stripes assembled and digest-checked, and the full
    host-pointer mpfft_mul_multi (host packing, H2D, the multiply, D2H of the stripes)."""
    import torch
    depth, w, nl = CONFIGS[cfg]
    G = len(devices)
    part = mp.shard_partition(nl, nl, depth, w, G)
    a = mp.fill_random(nl, SEED1)
    b = mp.fill_random(nl, SEED2)
    t0 = time.perf_counter()
    packs = [(mp.shard_pack(a, nl, nl, depth, w, G, g), mp.shard_pack(b, nl, nl, depth, w, G, g)) for g in range(G)]
    pack_ms = (time.perf_counter() - t0) * 1e3
    devs = [torch.device("cuda", d) for d in devices]
    src1 = [torch.from_numpy(packs[g][0].view(np.int64)).to(devs[g]) for g in range(G)]
    src2 = [torch.from_numpy(packs[g][1].view(np.int64)).to(devs[g]) for g in range(G)]
    del packs
    outs = [torch.empty(part["Tr"] * part["SL"], dtype=torch.int64, device=devs[g]) for g in range(G)]
    streams = [torch.cuda.Stream(device=devs[g]) for g in range(G)]

    def sync():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)
    for _ in range(warmup):
        mp.mul_multi_device(nl, nl, depth, w, devices, src1, src2, outs, streams=streams)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        mp.mul_multi_device(nl, nl, depth, w, devices, src1, src2, outs, streams=streams)
    sync()
    el = time.perf_counter() - t0
    exact = None
    if check:
        prod = mp.assemble_stripes(part, G, [o.cpu().numpy().view(np.uint64) for o in outs])
        want = golden_digest(cfg)
        exact = hashlib.sha256(prod.tobytes()).hexdigest() == want if want else None
        del prod
    del src1, src2, outs
    host_ms = None
    if host_reps > 0:
        mp.mul_multi(a, b, depth, w, devices)               # warm the host-pointer buffers
        t1 = time.perf_counter()
        for _ in range(host_reps):
            r = mp.mul_multi(a, b, depth, w, devices)
        host_ms = (time.perf_counter() - t1) / host_reps * 1e3
        if check and exact is not None:
            exact = exact and hashlib.sha256(r.tobytes()).hexdigest() == golden_digest(cfg)
        del r
    mp.multi_release()
    torch.cuda.empty_cache()
    shared = len(set(devices)) < G
    return {"config": cfg, "path": "mpfft_mul_multi_device (one process, per-rank streams, peer copies)",
            "devices": list(devices), "n_ranks": G, "steps": steps, "ms_per_step": el / steps * 1e3,
            "value": 2 * nl * steps / el, "unit": "limbs/s", "exact": exact,
            "host_pointer_ms": host_ms, "host_pack_ms_python": pack_ms,
            "note": ("ranks sharing a device: a rehearsal of the multi-GPU schedule, not a scaling point"
                     if shared else "device-resident operand slices; host_pointer_ms is the full mpfft_mul_multi "
                                    "call (its own threaded packing, H2D, multiply, D2H of the stripes)")}


def c_entry_child(cfg, G, share, steps, check, timeout=400):
    """Rank 0's C-entry sub-record from a child process (`--mode multi`, no torch.distributed
    environment): the cross-device peer path of mpfft_mul_multi has not run on separate GPUs
    before a multi-GPU node takes it, so a fault or a hang there ends the child, not the rank
    that prints the line."""
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}
    cmd = [sys.executable, os.path.abspath(__file__), "--mode", "multi", "--config", cfg, "--multi-ranks", str(G),
           "--steps", str(steps), "--warmup", "1", "--e2e-reps", "1"]
    cmd += (["--multi-share"] if share else []) + ([] if check else ["--no-check"])
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"the C entry did not finish within {timeout} s (child killed)"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"child exit status {p.returncode}", "stderr_tail": p.stderr[-800:]}
    return json.loads(lines[-1])


def c_entry_fallback_line(args, cfg, world, c_entry, err):
    """The N > 1 line when sharded.py raised on rank 0: the same C4 product over the same N
    devices through the one-process C entry (mpfft_mul_multi_device), with the failure named."""
    depth, w, nl = CONFIGS[cfg]
    ok = isinstance(c_entry, dict) and "value" in c_entry
    return {"metric": METRIC, "value": c_entry["value"] if ok else None, "unit": "limbs/s", "n_gpus": world,
            "steps": c_entry.get("steps") if ok else 0, "warmup": 1,
            "ms_per_step": c_entry["ms_per_step"] if ok else None, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (xoshiro256** limbs, seeds 0x1001/0x2002)",
            "config": {"workload": f"{cfg}: new_mpn_mul depth={depth} w={w} n1=n2={nl} limbs over {world} devices",
                       "parallelism": f"MFA columns x{world} through the one-process C entry (torch.distributed run failed)"},
            "exact": c_entry.get("exact") if ok else None, "sharded_error": err, "c_entry": c_entry}


def golden_digest(cfg):
    p = os.path.join(ROOT, "tests", "golden", "products.json")
    try:
        with open(p) as f:
            return {c["name"]: c["sha256"] for c in json.load(f)}.get(cfg)
    except OSError:
        return None


def launch_ranks(args):
    """--gpus N without a torch.distributed environment: start N rank processes (no GPU
    has been touched in this process) and return their exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, choices=sorted(set(CONFIGS) | set(CONFIGS6)),
                    help="default: C3 at N = 1, C4 at N > 1 (M4: --mul6 only)")
    ap.add_argument("--mode", default=None, choices=["single", "replicas", "sharded", "multi"],
                    help="N > 1: sharded (default) or independent replicas; multi: the one-process C entry "
                         "mpfft_mul_multi_device alone over --multi-ranks devices")
    ap.add_argument("--multi-ranks", type=int, default=0, help="--mode multi: ranks (devices 0 .. K-1)")
    ap.add_argument("--multi-share", action="store_true", help="--mode multi: every rank on device 0 (rehearsal)")
    ap.add_argument("--no-c-entry", action="store_true",
                    help="N > 1: skip rank 0's timing of the one-process C entry over the same devices")
    ap.add_argument("--cpu-reps", type=int, default=5, help="timed oracle calls (median; after one warm-up)")
    ap.add_argument("--cpu-warmup", type=int, default=1, help="untimed oracle calls before the timed ones")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="cpu_baseline.ncore: concurrent CPU multiplies (one process per core; 0: skip)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--e2e-reps", type=int, default=2)
    ap.add_argument("--no-twin", action="store_true",
                    help="skip the one-GPU C4 line (the N = 1 point of the sharded C4 curve)")
    ap.add_argument("--mul6", action="store_true",
                    help="time new_mpn_mul6 (sqrt2 front end) on --config C3 (default) or M4 instead")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rendezvous check without a GPU: every rank joins a gloo group and "
                         "rank 0 prints the world it saw (tests/test_bench_launcher.py)")
    args = ap.parse_args()

    if args.config and (args.config not in (CONFIGS6 if args.mul6 else CONFIGS)):
        ap.error(f"--config {args.config} is not a {'--mul6 ' if args.mul6 else ''}configuration")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        import torch
        import torch.distributed as dist
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            seen = int(t.item())
            if dist.get_rank() == 0:
                print(json.dumps({"n_gpus": world, "ranks_seen": seen, "dry_run": True}))
            dist.destroy_process_group()
        else:
            print(json.dumps({"n_gpus": 1, "ranks_seen": 1, "dry_run": True}))
        return

    # the multi-core CPU figure first: its worker processes start before anything touches the GPU
    ncore = None
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu_baseline and not args.mul6 \
            and args.mode in (None, "single") and args.cpu_procs > 0:
        ncore = cpu_ncore(args.config or "C3", args.cpu_procs)

    import torch
    import torch.distributed as dist
    import mpfft_loader
    mp = mpfft_loader.load()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = args.mode or ("sharded" if world > 1 else "single")
    cfg = args.config or ("C4" if world > 1 else "C3")
    # MPFFT_BENCH_SHARE_GPU=1 (rehearsal on a one-GPU box, not a measurement): every rank on
    # cuda:0 and gloo with host-staged exchanges -- the launcher and the sharded pipeline end
    # to end without RCCL (which does not run two ranks on one device)
    share = os.environ.get("MPFFT_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # A failure on some ranks only (an OOM partway through the sharded run) would leave the
        # others blocked inside an RCCL collective that the failed rank never joins, short of the
        # gloo barrier below where rank 0 falls back to the C entry's line.  Bounded waits turn that
        # into a symmetric failure: the RCCL group times out after 240 s and, with
        # TORCH_NCCL_ASYNC_ERROR_HANDLING=2 (clean up, do not tear the process down), the blocked
        # collective raises on those ranks too; the gloo group's barriers wait up to 900 s.  (The
        # symmetric case is rehearsed with MPFFT_BENCH_FAIL_SHARDED=1; the asymmetric one needs
        # distinct GPUs and has not run.)
        import datetime
        if share:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=900))
        else:
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=240))

    if args.mul6:
        print(json.dumps(bench_mul6(args, mp, dev, args.config or "C3")))
        return

    if mode == "sharded":
        from importlib import import_module
        sh = import_module("mpir_fft_amd.sharded")
        twin = None
        if rank == 0 and not args.no_twin:   # the same product on one GPU, same run
            twin = single_gpu_line(mp, dev, cfg, 3, 1, check=not args.no_check)
        if world > 1:
            dist.barrier()
        try:
            if os.environ.get("MPFFT_BENCH_FAIL_SHARDED") == "1":   # rehearsal of the fallback below
                raise RuntimeError("MPFFT_BENCH_FAIL_SHARDED=1")
            res, sharded_err = sh.bench(args, cfg, CONFIGS[cfg], rank, world, dev), None
        except Exception as e:   # reported on the line; rank 0 then falls back to the C entry's curve
            res, sharded_err = None, repr(e)
        # the other ranks wait on a host-side (gloo) barrier while rank 0 times the C entry on
        # their devices: an RCCL barrier would leave a kernel spinning on each of those GPUs
        host_pg = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=900)) if world > 1 else None
        if world > 1:
            dist.barrier(group=host_pg)
        if rank == 0:
            c_entry = None
            if not args.no_c_entry or res is None:
                # the same product through the one-process C entry over devices 0 .. N-1 (the
                # other ranks wait at the barrier below): a transport failure in one driver still
                # leaves a curve from the other
                torch.cuda.empty_cache()
                c_entry = c_entry_child(cfg, world, share, max(1, min(args.steps, 3)), not args.no_check)
            if res is None:   # the torch.distributed run failed on this rank: the C entry's line
                res = c_entry_fallback_line(args, cfg, world, c_entry, sharded_err)
            else:
                res["c_entry"] = c_entry
            res["n1_twin"] = twin
            print(json.dumps(res))
        if world > 1:
            dist.barrier(group=host_pg)
            dist.destroy_process_group()
        return

    if mode == "multi":   # the one-process C entry alone (one-GPU box: --multi-ranks K on device 0)
        K = args.multi_ranks or 1
        devs = [0] * K if args.multi_share else list(range(K))
        print(json.dumps(multi_entry_line(mp, cfg, devs, args.steps, args.warmup, check=not args.no_check,
                                          host_reps=args.e2e_reps)))
        return

    depth, w, nl = CONFIGS[cfg]
    n1 = n2 = nl
    P = mp.plan_info(n1, n2, depth, w)
    kern = mp.stage_kernels(n1, n2, depth, w)
    a = mp.fill_random(n1, SEED1 + 0x10000 * rank)
    b = mp.fill_random(n2, SEED2 + 0x10000 * rank)
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace(n1, n2, depth, w, dev)
    stream = torch.cuda.Stream(device=dev)

    def step():
        mp.mul_device(dr, da, n1, db, n2, depth, w, ws, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # timed region: K whole multiplies, one library call each, nothing else on the stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # stage breakdown: K more multiplies in which the library records a HIP event on its own
    # stream at every stage boundary (mpfft_profile_begin) -- kept out of the timed loop above
    torch.cuda.synchronize(dev)
    mp.profile_begin(args.steps)
    tp = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    prof_ms = (time.perf_counter() - tp) / args.steps * 1e3
    stage_tot, calls = mp.profile_end()
    stage_ms = {k: v / max(calls, 1) for k, v in stage_tot.items()}

    got = dr.cpu().numpy().view(np.uint64)
    exact = None
    if not args.no_check and rank == 0:
        want = golden_digest(cfg)
        if want is not None:
            exact = hashlib.sha256(got.tobytes()).hexdigest() == want

    # end to end through the drop-in boundary (host pointers: H2D, multiply, D2H)
    e2e = None
    if args.e2e_reps > 0 and rank == 0:
        r = np.zeros(n1 + n2, dtype=np.uint64)
        mp.new_mpn_mul(r, a, n1, b, n2, depth, w)          # warm the host-pointer context
        t1 = time.perf_counter()
        for _ in range(args.e2e_reps):
            mp.new_mpn_mul(r, a, n1, b, n2, depth, w)
        te = (time.perf_counter() - t1) / args.e2e_reps
        e2e = {"ms": te * 1e3, "limbs_per_s": (n1 + n2) / te, "same_product": bool((r == got).all()),
               "note": "host arrays: H2D of both operands, the multiply, D2H of the product (PCIe included)"}
        # the host link on its own (same pageable arrays; a pinned copy beside it): operand 1's H2D
        # cannot overlap the multiply (its first column pass reads the whole operand) and the
        # product's D2H cannot start before the combine, so h2d(i1) + device + d2h(r) bounds e2e
        ta, tr = torch.from_numpy(a), torch.from_numpy(r)
        dbuf = torch.empty(n1 + n2, dtype=torch.int64, device=dev)

        def rate(fn, nbytes, reps=3):
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return nbytes * reps / (time.perf_counter() - t) / 1e9

        h2d = rate(lambda: dbuf[:n1].copy_(ta.view(torch.int64)), n1 * 8)
        d2h = rate(lambda: tr.view(torch.int64).copy_(dbuf), (n1 + n2) * 8)
        pa, pr = ta.view(torch.int64).pin_memory(), tr.view(torch.int64).pin_memory()
        h2d_p = rate(lambda: dbuf[:n1].copy_(pa, non_blocking=True), n1 * 8)
        d2h_p = rate(lambda: pr.copy_(dbuf, non_blocking=True), (n1 + n2) * 8)
        # critical path of the host-pointer call (mpfft.hip mul_host): operand 1's H2D; then operand
        # 1's forward transform beside operand 2's H2D (copy stream); operand 2's forward transform;
        # the rest of the multiply; the product's D2H
        fwd1 = (stage_ms["fwd_columns"] + stage_ms["fwd_rows"]) / 2
        t_h1, t_h2, t_d = n1 * 8 / h2d * 1e-6, n2 * 8 / h2d * 1e-6, (n1 + n2) * 8 / d2h * 1e-6
        bound = t_h1 + max(t_h2, fwd1) + fwd1 + (el / args.steps * 1e3 - 2 * fwd1) + t_d
        e2e["link"] = {"h2d_pageable_GBs": h2d, "d2h_pageable_GBs": d2h, "h2d_pinned_GBs": h2d_p,
                       "d2h_pinned_GBs": d2h_p, "bound_ms": bound,
                       "note": "bound = H2D(op1) + max(H2D(op2), fwd(op1)) + fwd(op2) + the rest of the "
                               "multiply + D2H(product), at the pageable rates measured here: operand 2's "
                               "H2D (longer than operand 1's forward transform) hides only partly, and "
                               "operand 2's forward transform waits for it"}
        del r, ta, tr, dbuf, pa, pr
        mp.lib().mpfft_release()

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_step = el / args.steps * 1e3
    value = world * (n1 + n2) * args.steps / el
    dname = max(stage_ms, key=stage_ms.get)
    roof = roofline(cfg, kern[dname], dname, stage_bytes(P, dname, n1, n2), stage_ms[dname])
    balg = b_alg(P, n1, n2)
    dev_ms = float(sum(stage_ms.values()))
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "limbs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "scaling_note": "bench.py --gpus N > 1 splits one C4 product over the N GPUs (strong scaling); "
                        "its N = 1 point is `c4_single` below (this line's value is C3, the largest "
                        "single-GPU configuration)",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (xoshiro256** limbs, seeds 0x1001/0x2002 per rank)",
        "config": {"workload": f"{cfg}: new_mpn_mul depth={depth} w={w} n1=n2={nl} limbs "
                               f"(l={P['l']} limbs/coeff, NC x NR = {P['NC']} x {P['NR']}, trunc={P['trunc']})",
                   "parallelism": f"replicas x{world}" if world > 1 else "single"},
        "roofline": roof,
        "pipeline": {"device_ms": dev_ms, "b_alg_bytes": balg, "hbm_frac_b_alg": balg / (dev_ms * 1e-3) / HBM_PEAK,
                     "note": "whole multiply vs the HBM roofline of the three-pass MFA (SURVEY 8d)"},
        "stages_ms": stage_ms,
        "profiled_ms_per_step": prof_ms,
        "stage_kernels": kern,
        "e2e_host": e2e,
        "exact": exact,
        "exact_check": "SHA-256 of the product limbs vs tests/golden/products.json (GMP mpn_mul)",
    }
    if world == 1 and not args.no_twin and cfg != "C4":
        del dr, ws
        torch.cuda.empty_cache()
        res["c4_single"] = single_gpu_line(mp, dev, "C4", 3, 1, check=not args.no_check)
    if world == 1 and not args.no_cpu_baseline:
        cb, ref, g = cpu_baseline(a, b, depth, w, args.cpu_reps, args.cpu_warmup)
        cb["ncore"] = ncore
        res["cpu_baseline"] = cb
        res["exact_vs_port"] = bool((got == ref).all())
        res["exact_vs_gmp"] = bool((got == g).all())
    print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


def bench_mul6(args, mp, dev, cfg):
    """One-GPU line for new_mpn_mul6 (not the headline): device-resident multiplies timed
    like the main bench, exactness against the golden digest of the same operands."""
    import torch
    depth, w, nl = CONFIGS6[cfg]
    n1 = n2 = nl
    P = mp.plan_info6(n1, n2, depth, w)
    a = mp.fill_random(n1, SEED1)
    b = mp.fill_random(n2, SEED2)
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=dev)
    ws = mp.alloc_workspace6(n1, n2, depth, w, dev)
    stream = torch.cuda.Stream(device=dev)
    for _ in range(args.warmup):
        mp.mul6_device(dr, da, n1, db, n2, depth, w, ws, stream=stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mp.mul6_device(dr, da, n1, db, n2, depth, w, ws, stream=stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    got = dr.cpu().numpy().view(np.uint64)
    want = golden_digest(cfg) if cfg in CONFIGS and CONFIGS[cfg][2] == nl else None
    exact = hashlib.sha256(got.tobytes()).hexdigest() == want if want else None
    balg = b_alg(P, n1, n2)
    ms = el / args.steps * 1e3
    return {"metric": METRIC, "value": (n1 + n2) * args.steps / el, "unit": "limbs/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (xoshiro256** limbs, seeds 0x1001/0x2002)",
            "config": {"workload": f"{cfg} operands via new_mpn_mul6 depth={depth} w={w} n1=n2={nl} limbs "
                                   f"(l={P['l']}, 4n = {4 * P['n']} slots, trunc={P['trunc']})",
                       "parallelism": "single", "entry": "new_mpn_mul6 (sqrt2, mul_fft.c:3573)"},
            "pipeline": {"b_alg_bytes": balg, "hbm_frac_b_alg": balg / (ms * 1e-3) / HBM_PEAK},
            "exact": exact, "exact_check": "SHA-256 vs the new_mpn_mul golden digest of the same operands"}


if __name__ == "__main__":
    main()
