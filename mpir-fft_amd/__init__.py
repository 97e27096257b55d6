"""mpir-fft_amd -- MI355X-native drop-in for wbhart/mpir-fft's new_mpn_mul.

Host-side mirror of the reference interface for the hot path:

    new_mpn_mul(r1, i1, n1, i2, n2, depth, w)      # /root/reference/mul_fft.c:3190

same names, same argument meaning (little-endian 64-bit limb arrays, convolution
length 2^(depth+1) over Z/(2^(2^depth * w) + 1)), computed by the hand-written
HIP kernels in csrc/ through the C ABI of libmpfft.so (include/mpfft.h).

There is no CPU fallback: if libmpfft.so is missing or no GPU is visible, every
compute entry point raises.  Errors the reference would turn into a segfault
(mul_fft.c:3186-3188) raise MpfftError with the library's reason.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPFFT_LIB=diag selects the diagnostic build libmpfft_diag.so (make DIAG=1: tuning and
# ablation knobs for scripts/; never used by the tests, smoke() or the bench)
_LIBSEL = os.environ.get("MPFFT_LIB", "")
LIB_PATH = os.path.join(_HERE, "libmpfft_diag.so" if _LIBSEL == "diag" else
                        _LIBSEL if _LIBSEL.endswith(".so") else "libmpfft.so")   # a path: A/B scripts
_lib = None

STAGE_FWD_COLUMNS, STAGE_FWD_ROWS, STAGE_POINTWISE, STAGE_INV_ROWS, STAGE_INV_COLUMNS, \
    STAGE_SCALE, STAGE_COMBINE, STAGE_FOLD_COMBINE = range(8)

_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_L = ctypes.c_long
_UL = ctypes.c_ulong


class _Shard(ctypes.Structure):
    """struct mpfft_shard (include/mpfft.h)"""
    _fields_ = [("n1", ctypes.c_long), ("n2", ctypes.c_long), ("depth", ctypes.c_ulong), ("w", ctypes.c_ulong),
                ("c0", ctypes.c_int), ("ccount", ctypes.c_int), ("r0", ctypes.c_int), ("rcount", ctypes.c_int),
                ("ccb", ctypes.c_int),
                ("col_dig", ctypes.c_void_p * 2), ("col_cb", ctypes.c_void_p * 2), ("col_top", ctypes.c_void_p * 2),
                ("row_dig", ctypes.c_void_p * 2), ("row_cb", ctypes.c_void_p * 2), ("row_top", ctypes.c_void_p * 2),
                ("src_chunk", ctypes.c_long),
                ("rowc_dig", ctypes.c_void_p), ("rowc_cb", ctypes.c_void_p), ("rowc_top", ctypes.c_void_p)]


class _Copy(ctypes.Structure):
    """struct mpfft_copy (include/mpfft.h)"""
    _fields_ = [("src", ctypes.c_int), ("dst", ctypes.c_int), ("op", ctypes.c_int), ("field", ctypes.c_int),
                ("src_layout", ctypes.c_int), ("dst_layout", ctypes.c_int),
                ("src_off", ctypes.c_long), ("dst_off", ctypes.c_long), ("count", ctypes.c_long)]


XCHG_COL_TO_ROW, XCHG_ROW_TO_COL = 1, 2
LAYOUT_HALO = 2      # mpfft_copy.dst_layout of a halo copy


class MpfftError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: {strerror(code)} (code {code})")
        self.code = code


def lib():
    """The loaded libmpfft.so (raises if it was not built -- no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME,
        # different file name).  Loading torch first makes libmpfft's NEEDED
        # libamdhip64.so.7 bind to that copy, so device pointers and streams from
        # torch are valid here; loading libmpfft first would pull in /opt/rocm's copy
        # and a later torch import would start a second runtime that sees no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        h = ctypes.CDLL(LIB_PATH)
        h.new_mpn_mul.argtypes = [_u64p, _u64p, _L, _u64p, _L, _UL, _UL]
        h.new_mpn_mul.restype = None
        h.mpfft_mul_ex.argtypes = [_u64p, _u64p, _L, _u64p, _L, _UL, _UL]
        h.mpfft_mul_ex.restype = ctypes.c_int
        h.mpfft_profile_begin.argtypes = [ctypes.c_int]
        h.mpfft_profile_begin.restype = ctypes.c_int
        h.mpfft_profile_end.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
        h.mpfft_profile_end.restype = ctypes.c_int
        h.mpfft_stage_kernels.argtypes = [_L, _L, _UL, _UL, ctypes.c_char_p, ctypes.c_size_t]
        h.mpfft_stage_kernels.restype = ctypes.c_int
        h.mpfft_release.argtypes = []
        h.mpfft_release.restype = ctypes.c_int
        h.mpfft_mul_device.argtypes = [_vp, _vp, _L, _vp, _L, _UL, _UL, _vp, ctypes.c_size_t, _vp]
        h.mpfft_mul_device.restype = ctypes.c_int
        h.mpfft_stage.argtypes = [ctypes.c_int, _vp, _vp, _vp, _L, _L, _UL, _UL, _vp, ctypes.c_size_t, _vp]
        h.mpfft_stage.restype = ctypes.c_int
        h.mpfft_workspace_bytes.argtypes = [_L, _L, _UL, _UL]
        h.mpfft_workspace_bytes.restype = ctypes.c_size_t
        h.mpfft_check_params.argtypes = [_L, _L, _UL, _UL]
        h.mpfft_check_params.restype = ctypes.c_int
        h.mpfft_plan_info.argtypes = [_L, _L, _UL, _UL, ctypes.POINTER(ctypes.c_long)]
        h.mpfft_plan_info.restype = ctypes.c_int
        h.mpfft_workspace_layout.argtypes = [_L, _L, _UL, _UL, ctypes.POINTER(ctypes.c_size_t)]
        h.mpfft_workspace_layout.restype = ctypes.c_int
        h.mpfft_strerror.argtypes = [ctypes.c_int]
        h.mpfft_strerror.restype = ctypes.c_char_p
        h.mpfft_version.argtypes = []
        h.mpfft_version.restype = ctypes.c_int
        h.mpfft_fill_random.argtypes = [_u64p, _L, ctypes.c_uint64]
        h.mpfft_fill_random.restype = None
        h.mpfft_shard_stage.argtypes = [ctypes.c_int, ctypes.POINTER(_Shard), _vp, _vp, _vp]
        h.mpfft_shard_stage.restype = ctypes.c_int
        h.mpfft_shard_stage_rows.argtypes = [ctypes.c_int, ctypes.POINTER(_Shard), ctypes.c_int, ctypes.c_int, _vp]
        h.mpfft_shard_stage_rows.restype = ctypes.c_int
        h.mpfft_shard_row_fused.argtypes = [_L, _L, _UL, _UL, ctypes.c_int]
        h.mpfft_shard_row_fused.restype = ctypes.c_int
        h.mpfft_shard_combine_tmp_bytes.argtypes = [_L, _L, _UL, _UL, ctypes.c_int]
        h.mpfft_shard_combine_tmp_bytes.restype = ctypes.c_size_t
        h.mpfft_shard_combine.argtypes = [ctypes.POINTER(_Shard), ctypes.c_int, _vp, _vp, _vp, _vp, _vp,
                                          ctypes.c_size_t, _vp]
        h.mpfft_shard_combine.restype = ctypes.c_int
        _lp = ctypes.POINTER(ctypes.c_long)
        h.mpfft_shard_partition.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, _lp, _lp]
        h.mpfft_shard_partition.restype = ctypes.c_int
        h.mpfft_shard_stripes.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, _lp, _L]
        h.mpfft_shard_stripes.restype = ctypes.c_long
        h.mpfft_shard_exchange_plan.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(_Copy), _L]
        h.mpfft_shard_exchange_plan.restype = ctypes.c_long
        h.mpfft_shard_halo_plan.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, ctypes.POINTER(_Copy), _L]
        h.mpfft_shard_halo_plan.restype = ctypes.c_long
        h.mpfft_shard_src_limbs.argtypes = [_L, _L, _UL, _UL, ctypes.c_int]
        h.mpfft_shard_src_limbs.restype = ctypes.c_long
        h.mpfft_shard_pack.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, ctypes.c_int, _u64p, _L, _u64p]
        h.mpfft_shard_pack.restype = ctypes.c_int
        h.mpfft_mul_multi_device.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                             ctypes.POINTER(_vp)]
        h.mpfft_mul_multi_device.restype = ctypes.c_int
        h.mpfft_mul_multi.argtypes = [_u64p, _u64p, _L, _u64p, _L, _UL, _UL, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int)]
        h.mpfft_mul_multi.restype = ctypes.c_int
        h.mpfft_multi_release.argtypes = []
        h.mpfft_multi_release.restype = ctypes.c_int
        if hasattr(h, "mpfft_multi_schedule"):   # (older libraries in A/B runs lack it)
            h.mpfft_multi_schedule.argtypes = [_L, _L, _UL, _UL, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                               ctypes.c_size_t]
            h.mpfft_multi_schedule.restype = ctypes.c_long
        h.mpfft_set_devices.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), _L]
        h.mpfft_set_devices.restype = ctypes.c_int
        h.mpfft_last_ngpus.argtypes = []
        h.mpfft_last_ngpus.restype = ctypes.c_int
        h.mpfft_choose.argtypes = [_L, _L, ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_ulong)]
        h.mpfft_choose.restype = ctypes.c_int
        h.mpfft_mul_auto.argtypes = [_u64p, _u64p, _L, _u64p, _L]
        h.mpfft_mul_auto.restype = ctypes.c_int
        h.new_mpn_mul6.argtypes = [_u64p, _u64p, _L, _u64p, _L, _UL, _UL]
        h.new_mpn_mul6.restype = None
        h.mpfft_mul6_ex.argtypes = [_u64p, _u64p, _L, _u64p, _L, _UL, _UL]
        h.mpfft_mul6_ex.restype = ctypes.c_int
        h.mpfft_mul6_device.argtypes = [_vp, _vp, _L, _vp, _L, _UL, _UL, _vp, ctypes.c_size_t, _vp]
        h.mpfft_mul6_device.restype = ctypes.c_int
        h.mpfft_workspace_bytes6.argtypes = [_L, _L, _UL, _UL]
        h.mpfft_workspace_bytes6.restype = ctypes.c_size_t
        h.mpfft_check_params6.argtypes = [_L, _L, _UL, _UL]
        h.mpfft_check_params6.restype = ctypes.c_int
        h.mpfft_plan_info6.argtypes = [_L, _L, _UL, _UL, ctypes.POINTER(ctypes.c_long)]
        h.mpfft_plan_info6.restype = ctypes.c_int
        _lib = h
    return _lib


def strerror(code):
    return lib().mpfft_strerror(int(code)).decode()


def _p(a):
    if a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("limb arrays must be C-contiguous numpy.uint64")
    return a.ctypes.data_as(_u64p)


def check_params(n1, n2, depth, w):
    return lib().mpfft_check_params(n1, n2, depth, w)


def plan_info(n1, n2, depth, w):
    """dict of the derived parameters (mul_fft.c:3193-3203) or MpfftError."""
    out = (ctypes.c_long * 10)()
    rc = lib().mpfft_plan_info(n1, n2, depth, w, out)
    if rc:
        raise MpfftError(rc, f"plan(n1={n1}, n2={n2}, depth={depth}, w={w})")
    keys = ("n", "l", "NC", "j1", "j2", "trunc", "bits1", "NR", "tpb", "U")
    return dict(zip(keys, list(out)))


def workspace_bytes(n1, n2, depth, w):
    return int(lib().mpfft_workspace_bytes(n1, n2, depth, w))


def new_mpn_mul(r1, i1, n1, i2, n2, depth, w):
    """Reference-shaped entry (mul_fft.c:3190): r1[:n1+n2] = i1[:n1] * i2[:n2]."""
    if len(r1) < n1 + n2 or len(i1) < n1 or len(i2) < n2:
        raise ValueError("buffer shorter than the stated limb count")
    rc = lib().mpfft_mul_ex(_p(r1), _p(i1), n1, _p(i2), n2, depth, w)
    if rc:
        raise MpfftError(rc, f"new_mpn_mul(n1={n1}, n2={n2}, depth={depth}, w={w})")


def mul(i1, i2, depth, w):
    """Convenience: returns the n1+n2 limb product as a new uint64 array."""
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    new_mpn_mul(r, i1, len(i1), i2, len(i2), depth, w)
    return r


def choose(n1, n2):
    """(depth, w) the library would use for an n1 x n2-limb product (mpfft_choose: the
    reference leaves them to the caller, mul_fft.c:3190-3191)."""
    d, w = ctypes.c_ulong(), ctypes.c_ulong()
    rc = lib().mpfft_choose(n1, n2, ctypes.byref(d), ctypes.byref(w))
    if rc:
        raise MpfftError(rc, f"choose(n1={n1}, n2={n2})")
    return int(d.value), int(w.value)


def mul_auto(i1, i2):
    """mpn_mul-style product with (depth, w) from choose(): a new uint64 array of n1+n2 limbs."""
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    rc = lib().mpfft_mul_auto(_p(r), _p(i1), len(i1), _p(i2), len(i2))
    if rc:
        raise MpfftError(rc, f"mul_auto(n1={len(i1)}, n2={len(i2)})")
    return r


# ---- the sqrt2 front end (new_mpn_mul6, mul_fft.c:3573-3668) --------------------------

def check_params6(n1, n2, depth, w):
    return lib().mpfft_check_params6(n1, n2, depth, w)


def plan_info6(n1, n2, depth, w):
    """derived parameters of new_mpn_mul6 (mul_fft.c:3575-3603): bits1 = (N - depth - 1)/2,
    trunc over a length-4n convolution"""
    out = (ctypes.c_long * 10)()
    rc = lib().mpfft_plan_info6(n1, n2, depth, w, out)
    if rc:
        raise MpfftError(rc, f"plan6(n1={n1}, n2={n2}, depth={depth}, w={w})")
    keys = ("n", "l", "NC", "j1", "j2", "trunc", "bits1", "NR", "tpb", "U")
    return dict(zip(keys, list(out)))


def workspace_bytes6(n1, n2, depth, w):
    return int(lib().mpfft_workspace_bytes6(n1, n2, depth, w))


def new_mpn_mul6(r1, i1, n1, i2, n2, depth, w):
    """Reference-shaped entry (mul_fft.c:3573): r1[:n1+n2] = i1[:n1] * i2[:n2] through the
    sqrt2 transforms (length 4n, root sqrt2^w)"""
    if len(r1) < n1 + n2 or len(i1) < n1 or len(i2) < n2:
        raise ValueError("buffer shorter than the stated limb count")
    rc = lib().mpfft_mul6_ex(_p(r1), _p(i1), n1, _p(i2), n2, depth, w)
    if rc:
        raise MpfftError(rc, f"new_mpn_mul6(n1={n1}, n2={n2}, depth={depth}, w={w})")


def mul6(i1, i2, depth, w):
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    new_mpn_mul6(r, i1, len(i1), i2, len(i2), depth, w)
    return r


def alloc_workspace6(n1, n2, depth, w, device="cuda"):
    import torch
    nb = workspace_bytes6(n1, n2, depth, w)
    if nb == 0:
        raise MpfftError(check_params6(n1, n2, depth, w), "workspace6")
    return torch.empty(nb, dtype=torch.uint8, device=device)


def mul6_device(d_r, d_i1, n1, d_i2, n2, depth, w, ws, stream=None):
    """new_mpn_mul6 on HBM-resident operands; queued on `stream`, not synchronised."""
    rc = lib().mpfft_mul6_device(_ptr(d_r), _ptr(d_i1), n1, _ptr(d_i2), n2, depth, w, _ptr(ws),
                                 ws.numel() * ws.element_size(), _stream(stream))
    if rc:
        raise MpfftError(rc, "mpfft_mul6_device")


def fill_random(count, seed):
    buf = np.empty(count, dtype=np.uint64)
    lib().mpfft_fill_random(_p(buf), count, seed)
    return buf


# ---- device-resident entry points (torch tensors as HBM plumbing) ----------

def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def alloc_workspace(n1, n2, depth, w, device="cuda"):
    import torch
    nb = workspace_bytes(n1, n2, depth, w)
    if nb == 0:
        raise MpfftError(check_params(n1, n2, depth, w), "workspace")
    return torch.empty(nb, dtype=torch.uint8, device=device)


def mul_device(d_r, d_i1, n1, d_i2, n2, depth, w, ws, stream=None):
    """All tensors on the GPU (int64/uint64 limbs); queued on `stream`, not synchronised."""
    rc = lib().mpfft_mul_device(_ptr(d_r), _ptr(d_i1), n1, _ptr(d_i2), n2, depth, w, _ptr(ws),
                                ws.numel() * ws.element_size(), _stream(stream))
    if rc:
        raise MpfftError(rc, "mpfft_mul_device")


def stage(which, d_i1, d_i2, d_r, n1, n2, depth, w, ws, stream=None):
    rc = lib().mpfft_stage(which, _ptr(d_i1), _ptr(d_i2), _ptr(d_r), n1, n2, depth, w, _ptr(ws),
                           ws.numel() * ws.element_size(), _stream(stream))
    if rc:
        raise MpfftError(rc, f"mpfft_stage({which})")


STAGE_NAMES = ("fwd_columns", "fwd_rows", "pointwise", "inv_rows", "inv_columns", "scale", "combine")


def stage_kernels(n1, n2, depth, w):
    """dict stage -> the kernel the library launches for it with these parameters"""
    buf = ctypes.create_string_buffer(512)
    rc = lib().mpfft_stage_kernels(n1, n2, depth, w, buf, len(buf))
    if rc:
        raise MpfftError(rc, "mpfft_stage_kernels")
    return dict(zip(STAGE_NAMES, buf.value.decode().split(";")))


def profile_begin(max_calls):
    """Record HIP events at the stage boundaries of the next max_calls multiplies."""
    rc = lib().mpfft_profile_begin(max_calls)
    if rc:
        raise MpfftError(rc, "mpfft_profile_begin")


def profile_end():
    """(dict stage -> summed ms, number of profiled multiplies); synchronises."""
    ms = (ctypes.c_float * len(STAGE_NAMES))()
    calls = ctypes.c_int(0)
    rc = lib().mpfft_profile_end(ms, ctypes.byref(calls))
    if rc:
        raise MpfftError(rc, "mpfft_profile_end")
    return dict(zip(STAGE_NAMES, [float(x) for x in ms])), calls.value


def workspace_layout(n1, n2, depth, w):
    out = (ctypes.c_size_t * 8)()
    rc = lib().mpfft_workspace_layout(n1, n2, depth, w, out)
    if rc:
        raise MpfftError(rc, "workspace_layout")
    keys = ("digA", "topA", "cbA", "digB", "topB", "cbB", "slots", "cbw")
    return dict(zip(keys, list(out)))


def workspace_views(ws, n1, n2, depth, w):
    """(digA, topA, digB, topB) views into a single-GPU workspace tensor (slot-major).
    Only meaningful for canonically stored stages (carry masks zero)."""
    import torch
    P = plan_info(n1, n2, depth, w)
    lay = workspace_layout(n1, n2, depth, w)
    slots, l = lay["slots"], P["l"]
    u8 = ws.view(torch.uint8)

    def dig(off):
        return u8[off:off + slots * l * 8].view(torch.int64).view(slots, l)

    def top(off):
        return u8[off:off + slots * 4].view(torch.int32)
    return dig(lay["digA"]), top(lay["topA"]), dig(lay["digB"]), top(lay["topB"])


# ---- sharded (multi-GPU) stages: see sharded.py ------------------------------

def shard_desc(sh):
    """dict from sharded.ShardedMul.shard_desc() -> struct mpfft_shard"""
    d = _Shard()
    for k in ("n1", "n2", "depth", "w", "c0", "ccount", "r0", "rcount", "ccb"):
        setattr(d, k, int(sh[k]))
    for k in (0, 1):
        d.col_dig[k] = sh["col"][k]["dig"].data_ptr()
        d.col_cb[k] = sh["col"][k]["cb"].data_ptr()
        d.col_top[k] = sh["col"][k]["top"].data_ptr()
        d.row_dig[k] = sh["row"][k]["dig"].data_ptr()
        d.row_cb[k] = sh["row"][k]["cb"].data_ptr()
        d.row_top[k] = sh["row"][k]["top"].data_ptr()
    d.src_chunk = int(sh.get("src_chunk", 0))
    rc = sh.get("rowc")
    if rc is not None:
        d.rowc_dig, d.rowc_cb, d.rowc_top = rc["dig"].data_ptr(), rc["cb"].data_ptr(), rc["top"].data_ptr()
    return d


def shard_row_fused(n1, n2, depth, w, ccb):
    """True if the sharded row stages fuse the last row DIF level into the pointwise
    (the caller then supplies a third row-layout array, `rowc`)."""
    return bool(lib().mpfft_shard_row_fused(n1, n2, depth, w, ccb))


def shard_stage(which, desc, d_i1, d_i2, stream=None):
    rc = lib().mpfft_shard_stage(which, ctypes.byref(desc), _ptr(d_i1), _ptr(d_i2), _stream(stream))
    if rc:
        raise MpfftError(rc, f"mpfft_shard_stage({which})")


def shard_stage_rows(which, desc, lo, hi, stream=None):
    """The row stages (SHARD_FWD_ROWS / POINTWISE / INV_ROWS) on local rows [lo, hi) only."""
    rc = lib().mpfft_shard_stage_rows(which, ctypes.byref(desc), lo, hi, _stream(stream))
    if rc:
        raise MpfftError(rc, f"mpfft_shard_stage_rows({which}, {lo}, {hi})")


def shard_combine_tmp_bytes(n1, n2, depth, w, world):
    return int(lib().mpfft_shard_combine_tmp_bytes(n1, n2, depth, w, world))


def shard_combine(desc, phase, d_r, halo, d_sums, d_sums_all, tmp, stream=None):
    """The rank's product stripes from its column layout (include/mpfft.h mpfft_shard_combine):
    phase 0 with carry-in 0 + stripe summaries into d_sums, phase 1 the carries from d_sums_all."""
    rc = lib().mpfft_shard_combine(ctypes.byref(desc), phase, _ptr(d_r), _ptr(halo), _ptr(d_sums), _ptr(d_sums_all),
                                   _ptr(tmp), tmp.numel(), _stream(stream))
    if rc:
        raise MpfftError(rc, f"mpfft_shard_combine(phase {phase})")


# ---- multi-GPU from one process (mpfft_mul_multi, multi.hip) ------------------------

def shard_partition(n1, n2, depth, w, world):
    """The C partition of one column-sharded multiply: dict rows (list of world + 1), C, chunk,
    H, Tr, fused, SL, S, ms (the stripes' first product limbs, S + 1) (mpfft_shard_partition,
    mpfft_shard_stripes)."""
    rows = (ctypes.c_long * (world + 1))()
    info = (ctypes.c_long * 7)()
    rc = lib().mpfft_shard_partition(n1, n2, depth, w, world, rows, info)
    if rc:
        raise MpfftError(rc, f"shard_partition(world={world})")
    S = info[6]
    ms = (ctypes.c_long * (S + 1))()
    n = lib().mpfft_shard_stripes(n1, n2, depth, w, world, ms, S + 1)
    if n != S + 1:
        raise MpfftError(-n if n < 0 else 1, "shard_stripes")
    return {"rows": list(rows), "C": info[0], "chunk": info[1], "H": info[2], "Tr": info[3],
            "fused": bool(info[4]), "SL": info[5], "S": S, "ms": list(ms)}


def _copies(fn, *args):
    n = fn(*args, None, 0)
    if n < 0:
        raise MpfftError(-n, fn.__name__)
    out = (_Copy * max(n, 1))()
    n = fn(*args, out, n)
    if n < 0:
        raise MpfftError(-n, fn.__name__)
    return [{f: getattr(out[i], f) for f, _ in _Copy._fields_} for i in range(n)]


def shard_exchange_plan(n1, n2, depth, w, world, which):
    """The copies of exchange `which` (XCHG_*): list of dicts (mpfft_shard_exchange_plan)."""
    return _copies(lib().mpfft_shard_exchange_plan, n1, n2, depth, w, world, which)


def shard_halo_plan(n1, n2, depth, w, world):
    """The halo copies before the combine (mpfft_shard_halo_plan): column layout -> halo, limbs."""
    return _copies(lib().mpfft_shard_halo_plan, n1, n2, depth, w, world)


def shard_src_limbs(n1, n2, depth, w, world):
    n = lib().mpfft_shard_src_limbs(n1, n2, depth, w, world)
    if n < 0:
        raise MpfftError(-n, "shard_src_limbs")
    return n


def shard_pack(a, n1, n2, depth, w, world, rank):
    """rank's operand slices of operand `a` (uint64 limbs), as the device-resident multi-GPU
    entry and the sharded drivers read them (mpfft_shard_pack)."""
    a = np.ascontiguousarray(a, dtype=np.uint64)
    out = np.empty(shard_src_limbs(n1, n2, depth, w, world), dtype=np.uint64)
    rc = lib().mpfft_shard_pack(n1, n2, depth, w, world, rank, _p(a), len(a), _p(out))
    if rc:
        raise MpfftError(rc, "shard_pack")
    return out


def mul_multi_device(n1, n2, depth, w, devices, src1, src2, outs, streams=None):
    """Device-resident multi-GPU multiply (mpfft_mul_multi_device): src1[g], src2[g] rank g's
    packed slices on devices[g] (torch tensors), outs[g] its Tr * SL stripe limbs.  streams:
    torch streams per rank (the work is ordered on them), or None (returns when done)."""
    G = len(devices)
    devs = (ctypes.c_int * G)(*devices)
    P = (_vp * G)
    s1 = P(*[t.data_ptr() for t in src1])
    s2 = P(*[t.data_ptr() for t in src2])
    r = P(*[t.data_ptr() for t in outs])
    st = P(*[s.cuda_stream for s in streams]) if streams is not None else None
    rc = lib().mpfft_mul_multi_device(n1, n2, depth, w, G, devs, s1, s2, r, st)
    if rc:
        raise MpfftError(rc, f"mul_multi_device(devices={list(devices)})")


def assemble_stripes(part, world, stripes):
    """The product from every rank's stripe buffers (stripes[g]: Tr * SL limbs, uint64)."""
    ms, SL = part["ms"], part["SL"]
    out = np.empty(ms[-1], dtype=np.uint64)
    for s in range(len(ms) - 1):
        g, j = s % world, s // world
        n = ms[s + 1] - ms[s]
        out[ms[s]: ms[s + 1]] = stripes[g][j * SL: j * SL + n]
    return out


def mul_multi(i1, i2, depth, w, devices):
    """r = i1 * i2 column-sharded over len(devices) ranks (devices may repeat), one process."""
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    devs = (ctypes.c_int * len(devices))(*devices)
    rc = lib().mpfft_mul_multi(_p(r), _p(i1), len(i1), _p(i2), len(i2), depth, w, len(devices), devs)
    if rc:
        raise MpfftError(rc, f"mul_multi(devices={list(devices)})")
    return r


def set_devices(devices, min_l=0):
    """new_mpn_mul policy: shard products with >= min_l-limb coefficients over `devices`."""
    devs = (ctypes.c_int * max(len(devices), 1))(*devices)
    return lib().mpfft_set_devices(len(devices), devs, min_l)


def multi_release():
    return lib().mpfft_multi_release()


def multi_schedule(n1, n2, depth, w, world, calls=1):
    """The event graph of `calls` back-to-back device-resident multi-rank multiplies
    (mpfft_multi_schedule: a dry run, no GPU): list of (kind, rank, stream, *rest) tuples."""
    n = lib().mpfft_multi_schedule(n1, n2, depth, w, world, calls, None, 0)
    if n < 0:
        raise MpfftError(-n, "multi_schedule")
    buf = ctypes.create_string_buffer(n)
    lib().mpfft_multi_schedule(n1, n2, depth, w, world, calls, buf, n)
    out = []
    for line in buf.value.decode().splitlines():
        f = line.split()
        out.append(tuple([f[0]] + [int(x) if x.lstrip("-").isdigit() else x for x in f[1:]]))
    return out
