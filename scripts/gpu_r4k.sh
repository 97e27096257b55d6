#!/bin/bash
# round 4, call K: C2 / C3 with the shipped library, libmpfft_fwd4.so (four-level l = 2048
# forward passes, 256 x 256 split) and libmpfft_fwd4f.so (same + fused row side): kernel
# statistics and two timed bench runs each
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for c in C2 C3; do
  for v in main fwd4 fwd4f; do
    if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks4_${c}_$v -o c -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/ks4_${c}_$v.log 2>&1 || exit 1
    echo "== $c $v"; python3 scripts/kstats.py gpurun_out/ks4_${c}_$v 14
    for r in 1 2; do
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-twin > gpurun_out/ab4_${c}_${v}_$r.log 2>&1 || exit 1
    done
  done
done
