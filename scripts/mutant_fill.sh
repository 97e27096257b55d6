#!/bin/bash
# Build a mutant libmpfft with a reconstructed round-3 FILL-fold defect: rp_store adds the
# pair-overflow carry into the coefficient registers in place, so the FILL step's second,
# rotated store (k_rpass DIT mode bit 2) starts from already-carried limbs.  Used only to
# show that tests/test_gpu_parity.py::test_fill_fold_l4096_case_b catches that defect.
# Output: mpir-fft_amd/libmpfft_mutfill.so (built from a copy under /tmp; csrc/ untouched).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/mpfft_mutfill
rm -rf $T && mkdir -p $T/mpir-fft_amd $T/include
cp -r $ROOT/mpir-fft_amd/csrc $T/mpir-fft_amd/ && cp $ROOT/include/mpfft.h $T/include/
rm -rf $T/mpir-fft_amd/csrc/build*
python3 - $T/mpir-fft_amd/csrc/rkernels.hpp <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
a = "__device__ __forceinline__ void rp_store(const Pr (&x)[NSX][rp_r(PP, NT)]"
b = "            u32 w0 = x[i][r].w[0], w1 = x[i][r].w[1];   // x itself stays intact (k_rpass FILL stores it twice)\n            add_small(w0, w1, hin, k0);"
assert a in s and b in s
s = s.replace(a, "__device__ __forceinline__ void rp_store(Pr (&x)[NSX][rp_r(PP, NT)]")
s = s.replace(b, "            add_small(x[i][r].w[0], x[i][r].w[1], hin, k0);   // MUTANT: in place\n            u32 w0 = x[i][r].w[0], w1 = x[i][r].w[1];")
open(p, "w").write(s)
PY
make -s -C $T/mpir-fft_amd/csrc -j8 >/dev/null
cp $T/mpir-fft_amd/libmpfft.so $ROOT/mpir-fft_amd/libmpfft_mutfill.so
echo "built $ROOT/mpir-fft_amd/libmpfft_mutfill.so"
