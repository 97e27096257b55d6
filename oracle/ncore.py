"""TEST INFRASTRUCTURE ONLY -- the host's multi-core capacity for the bench's cpu_baseline.

K independent processes, each pinned to its own core, run the CPU new_mpn_mul (oracle/, the
restatement of mul_fft.c:3190) -- and then GMP mpn_mul -- on the same operands at the same time;
the aggregate rate is K (n1 + n2) limbs over the wall time from the common start to the last
finish ("optionally the nproc-way throughput").  Run by bench.py before it touches
the GPU (the workers are plain Python + ctypes processes; nothing here imports torch).

  python oracle/ncore.py --procs K --depth D --w W --n N --seed1 S1 --seed2 S2   -> one JSON line
"""
import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def worker(args):
    sys.path.insert(0, HERE)
    import oracle as O
    os.sched_setaffinity(0, {args.core})
    a = O.fill_random(args.n, args.seed1)
    b = O.fill_random(args.n, args.seed2)
    sys.stdout.write("ready\n")
    sys.stdout.flush()
    sys.stdin.readline()   # the common start
    t0 = time.time()
    O.new_mpn_mul(a, b, args.depth, args.w)
    t1 = time.time()
    sys.stdout.write(f"mul {t0:.6f} {t1:.6f}\n")
    sys.stdout.flush()
    sys.stdin.readline()   # GMP together as well
    t2 = time.time()
    O.gmp_mul(a, b)
    t3 = time.time()
    sys.stdout.write(f"gmp {t2:.6f} {t3:.6f}\n")
    sys.stdout.flush()


def mem_available():
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def run(procs, depth, w, n, seed1, seed2, per_call_bytes):
    """K = min(procs, cores this process may run on, available RAM / per_call_bytes) workers"""
    cores = sorted(os.sched_getaffinity(0))
    mem = mem_available()
    k = max(1, min(procs, len(cores), int(mem * 0.8 // per_call_bytes) if mem else procs))
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--depth", str(depth), "--w", str(w),
           "--n", str(n), "--seed1", str(seed1), "--seed2", str(seed2)]
    ws = [subprocess.Popen(cmd + ["--core", str(cores[i])], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
          for i in range(k)]
    try:
        for p in ws:
            assert p.stdout.readline().strip() == "ready"
        res = {}
        for phase in ("mul", "gmp"):
            t0 = time.time()
            for p in ws:
                p.stdin.write("go\n")
                p.stdin.flush()
            ends = []
            for p in ws:
                f = p.stdout.readline().split()
                assert f and f[0] == phase, f
                ends.append(float(f[2]) - float(f[1]))
            wall = time.time() - t0
            res[phase] = (wall, ends)
        for p in ws:
            p.stdin.close()
            p.wait(timeout=60)
    finally:
        for p in ws:
            if p.poll() is None:
                p.kill()
    (wm, em), (wg, eg) = res["mul"], res["gmp"]
    limbs = 2 * n
    return {"value": k * limbs / wm, "unit": "limbs/s", "cores": k, "kind": "port",
            "sample": f"{k} concurrent full new_mpn_mul calls of the bench operands via oracle/ (one process per "
                      f"core, cores {cores[:k][0]}..{cores[:k][-1]}), {wm:.2f} s wall from the common start "
                      f"to the last finish (per call {min(em):.2f} .. {max(em):.2f} s)",
            "k_limit": {"requested": procs, "cores_allowed": len(cores), "mem_available_bytes": mem,
                        "per_call_bytes": per_call_bytes},
            "gmp_mpn_mul_limbs_per_s": k * limbs / wg, "gmp_mpn_mul_wall_s": wg}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--core", type=int, default=0)
    ap.add_argument("--depth", type=int, required=True)
    ap.add_argument("--w", type=int, required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--seed1", type=int, required=True)
    ap.add_argument("--seed2", type=int, required=True)
    ap.add_argument("--per-call-bytes", type=float, default=4e9)
    args = ap.parse_args()
    if args.worker:
        worker(args)
        return
    print(json.dumps(run(args.procs, args.depth, args.w, args.n, args.seed1, args.seed2, args.per_call_bytes)))


if __name__ == "__main__":
    main()
