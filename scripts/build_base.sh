#!/bin/bash
# Build libmpfft at a git revision (default HEAD) into mpir-fft_amd/libmpfft_base.so, for A/B
# runs of an uncommitted change against it (scripts/gpu_libab.sh ... libmpfft_base.so).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
T=/tmp/mpfft_base
rm -rf $T && mkdir -p $T
git -C $ROOT archive $REV mpir-fft_amd/csrc include | tar -x -C $T
make -s -C $T/mpir-fft_amd/csrc -j8 >/dev/null
cp $T/mpir-fft_amd/libmpfft.so $ROOT/mpir-fft_amd/libmpfft_base.so
echo "built libmpfft_base.so at $(git -C $ROOT rev-parse --short $REV)"
