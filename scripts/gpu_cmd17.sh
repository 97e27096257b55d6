# C1 tunable sweep: pass split (MPFFT_WLOGG) and k_pwm2 chain depth (MPFFT_PWM2_D4)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
for cfg in "" "MPFFT_WLOGG=4" "MPFFT_WLOGG=3" "MPFFT_PWM2_D4=1"; do
  echo "== $cfg" >> gpurun_out/sweep17.log
  env $cfg timeout -k 10 120 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/sweep17_tmp.log 2>&1 || exit $?
  tail -1 gpurun_out/sweep17_tmp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('exact'), d['stages_ms'])" >> gpurun_out/sweep17.log
done
cat gpurun_out/sweep17.log
