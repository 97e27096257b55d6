cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
for cfg in C3 C4; do for bl in 1 2 3; do
  if [ $cfg = C4 ] && [ $bl = 3 ]; then continue; fi
  echo "== $cfg BLOGG=$bl"; MPFFT_BLOGG=$bl timeout -k 10 200 python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-check | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: round(v,2) for k,v in d['stages_ms'].items()})" || exit 1
done; done > gpurun_out/sweep1.log 2>&1
