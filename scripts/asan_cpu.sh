#!/bin/bash
# SURVEY 5 "sanitizers": the CPU suite (-m "not gpu") against AddressSanitizer + UBSan builds of the
# host code -- libmpfft's planners / partition / copy, halo and schedule plans / argument checks
# (make -C mpir-fft_amd/csrc ASAN=1) and the oracle (make -C oracle asan) -- in one process with
# clang's sanitizer runtime preloaded.  Log: profiles/r06/asan_cpu.log (or $1).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$ROOT/profiles/r06/asan_cpu.log}
make -s -C $ROOT/mpir-fft_amd/csrc -j8 ASAN=1
make -s -C $ROOT/oracle asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n 1)
cd $ROOT
set +e
# leaks: the interpreter's own allocations are not ours to report
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  MPFFT_LIB=$ROOT/mpir-fft_amd/libmpfft_asan.so MPFFT_ORACLE_LIB=$ROOT/oracle/_asan/liboracle.so \
  python -m pytest tests -m "not gpu" -q -p no:cacheprovider > $LOG 2>&1
rc=$?
{ echo "# LD_PRELOAD=$(basename $RT) MPFFT_LIB=libmpfft_asan.so MPFFT_ORACLE_LIB=oracle/_asan/liboracle.so rc=$rc";
  echo "# sanitizer reports: $(grep -c 'ERROR: AddressSanitizer\|runtime error:' $LOG)"; } >> $LOG
tail -n 4 $LOG
exit $rc
