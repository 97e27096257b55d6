#!/bin/bash
# Round 5, call L: staggered first-round pointwise workgroups (PW_STAGGER A/B builds), pointwise
# stage alone at C3 and C4 shapes (scripts/pw_time.py), each library twice.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5l} && : > gpurun_out/pw_stagger_$T.log && \
for rep in 1 2; do for lib in libmpfft.so libmpfft_st3.so libmpfft_st6.so libmpfft_st12.so; do for c in C3 C4; do \
  echo -n "$lib " >> gpurun_out/pw_stagger_$T.log; \
  MPFFT_LIB=$GRAFT_REPO_ROOT/mpir-fft_amd/$lib timeout -k 10 120 python3 -u scripts/pw_time.py $c 10 >> gpurun_out/pw_stagger_$T.log 2>&1 || exit 1; \
done; done; done; cat gpurun_out/pw_stagger_$T.log
