"""Diagnostic: which HIP runtime does libmpfft bind to, with and without torch loaded first."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
if mode == "torch":
    import torch
    print("torch sees", torch.cuda.is_available(), torch.cuda.device_count())
import mpfft_loader
mp = mpfft_loader.load()
h = mp.lib()
hip = ctypes.CDLL("libamdhip64.so.7")
v = ctypes.c_int()
print("hipRuntimeGetVersion rc", hip.hipRuntimeGetVersion(ctypes.byref(v)), v.value)
cnt = ctypes.c_int()
print("hipGetDeviceCount rc", hip.hipGetDeviceCount(ctypes.byref(cnt)), cnt.value)
with open("/proc/self/maps") as f:
    libs = sorted({l.split()[-1] for l in f if "amdhip" in l or "hsa-runtime" in l})
print("\n".join(libs))
print({k: v for k, v in os.environ.items() if "VISIBLE" in k or "HSA" in k or "HIP" in k or "ROC" in k})
a = mp.fill_random(50, 1); b = mp.fill_random(40, 2)
r = np.zeros(90, np.uint64)
rc = h.mpfft_mul_ex(r.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 50,
                    b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 40, 8, 2)
print("mul_ex rc", rc, mp.strerror(rc))
A = int.from_bytes(a.tobytes(), "little"); B = int.from_bytes(b.tobytes(), "little")
print("exact:", int.from_bytes(r.tobytes(), "little") == A * B)
