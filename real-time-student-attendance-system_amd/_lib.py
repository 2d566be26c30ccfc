"""ctypes binding of libsketch.so (the C-ABI declared in include/sketch.h).

The library is built in-tree (``csrc/libsketch.so``) by
``__graft_entry__.build()``.  There is no fallback: if the library is missing
or no GPU can be opened, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SKE_LIB names another build of the same ABI (A/B timing of kernel variants;
# tools/ab_build.sh); the default is the in-tree build.
LIB_PATH = os.environ.get("SKE_LIB") or os.path.join(_HERE, "csrc", "libsketch.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "sketch.h")

SKE_OK = 0
SKE_EINVAL = -1
SKE_ENOMEM = -2
SKE_EHIP = -3
SKE_ENOFILTER = -4
SKE_EEXISTS = -5
SKE_EFULL = -6
SKE_ERANGE = -7
SKE_EBADRATE = -8
SKE_EBADCAP = -9
SKE_EBADEXP = -10
SKE_EBADHLL = -11
SKE_ETOOLONG = -12
SKE_EBUSY = -13
SKE_MEM_HOST = 0
SKE_MEM_DEVICE = 1
SKE_MAX_FILTERS = 4096
HLL_REGISTERS = 16384
HLL_DENSE_BYTES = 12288


class SketchLibError(RuntimeError):
    """libsketch returned an error code (carries the Redis-style text)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


class BfInfo(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("size_bytes", C.c_uint64), ("nfilters", C.c_uint32),
                ("expansion", C.c_uint32), ("inserted", C.c_uint64), ("nonscaling", C.c_int32),
                ("pad_", C.c_int32)]


class BfLink(C.Structure):
    _fields_ = [("entries", C.c_uint64), ("bytes", C.c_uint64), ("bits", C.c_uint64),
                ("size", C.c_uint64), ("error", C.c_double), ("bpe", C.c_double),
                ("hashes", C.c_int32), ("pad_", C.c_int32)]


class IngestCols(C.Structure):
    _fields_ = [("status", C.c_void_p), ("id_start", C.c_void_p), ("id_len", C.c_void_p),
                ("lec_start", C.c_void_p), ("lec_len", C.c_void_p), ("ts_start", C.c_void_p),
                ("ts_len", C.c_void_p), ("day", C.c_void_p), ("kh", C.c_void_p)]


class GenParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("id_lo", C.c_uint64), ("id_hi", C.c_uint64),
                ("n_members", C.c_uint64), ("perm_mul", C.c_uint64), ("perm_add", C.c_uint64),
                ("perm_mul_inv", C.c_uint64), ("invalid_thresh", C.c_uint32),
                ("near_thresh", C.c_uint32), ("n_keys", C.c_uint32), ("slot_base", C.c_uint32),
                ("key_cdf", C.c_void_p)]


_vp, _u8p, _u32p, _u64p = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
_CTX = C.c_void_p

# name -> (restype, argtypes); every symbol declared in include/sketch.h
SIGNATURES = {
    "ske_open": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "ske_close": (C.c_int, [_CTX]),
    "ske_strerror": (C.c_char_p, [C.c_int]),
    "ske_last_hip_error": (C.c_char_p, [_CTX]),
    "ske_set_stream": (C.c_int, [_CTX, _vp]),
    "ske_get_stream": (C.c_int, [_CTX, C.POINTER(_vp)]),
    "ske_sync": (C.c_int, [_CTX]),
    "ske_check_errors": (C.c_int, [_CTX]),
    "ske_device_alloc": (C.c_int, [_CTX, C.c_uint64, C.POINTER(C.c_void_p)]),
    "ske_device_free": (C.c_int, [_CTX, _vp]),
    "ske_memcpy": (C.c_int, [_CTX, _vp, _vp, C.c_uint64, C.c_int]),
    "ske_bf_reserve": (C.c_int, [_CTX, C.c_uint32, C.c_double, C.c_uint64, C.c_uint32, C.c_int]),
    "ske_bf_exists_key": (C.c_int, [_CTX, C.c_uint32]),
    "ske_bf_free": (C.c_int, [_CTX, C.c_uint32]),
    "ske_bf_madd": (C.c_int, [_CTX, C.c_uint32, _u8p, _u32p, C.c_uint64, _vp, C.c_int]),
    "ske_bf_mexists": (C.c_int, [_CTX, C.c_uint32, _u8p, _u32p, C.c_uint64, _u8p, C.c_int]),
    "ske_bf_info": (C.c_int, [_CTX, C.c_uint32, C.POINTER(BfInfo)]),
    "ske_bf_link_info": (C.c_int, [_CTX, C.c_uint32, C.c_uint32, C.POINTER(BfLink)]),
    "ske_bf_export_link": (C.c_int, [_CTX, C.c_uint32, C.c_uint32, _u8p, C.c_uint64]),
    "ske_bf_import_link": (C.c_int, [_CTX, C.c_uint32, C.c_uint32, _u8p, C.c_uint64]),
    "ske_bf_link_write": (C.c_int, [_CTX, C.c_uint32, C.c_uint32, C.c_uint64, _u8p, C.c_uint64]),
    "ske_bf_load_header": (C.c_int, [_CTX, C.c_uint32, C.POINTER(BfLink), C.c_uint32, C.c_uint64,
                                     C.c_uint32, C.c_int]),
    "ske_hll_reserve": (C.c_int, [_CTX, C.c_uint32]),
    "ske_hll_capacity": (C.c_uint32, [_CTX]),
    "ske_hll_clear": (C.c_int, [_CTX, C.c_uint32]),
    "ske_hll_pfadd": (C.c_int, [_CTX, _u32p, _u8p, _u32p, C.c_uint64, _u8p, C.c_int]),
    "ske_hll_pfcount": (C.c_int, [_CTX, _u32p, C.c_uint32, _u64p]),
    "ske_hll_pfcount_each": (C.c_int, [_CTX, _u32p, C.c_uint32, _u64p, C.c_int]),
    "ske_hll_pfcount_groups": (C.c_int, [_CTX, _u32p, _u32p, C.c_uint32, _u64p, C.c_int]),
    "ske_hll_pfmerge": (C.c_int, [_CTX, C.c_uint32, _u32p, C.c_uint32]),
    "ske_hll_pfmerge_dev": (C.c_int, [_CTX, C.c_uint32, _vp, C.c_uint32]),
    "ske_hll_histogram": (C.c_int, [_CTX, C.c_uint32, _u32p]),
    "ske_hll_export_raw": (C.c_int, [_CTX, C.c_uint32, _u8p]),
    "ske_hll_export_dense": (C.c_int, [_CTX, C.c_uint32, _u8p]),
    "ske_hll_import_raw": (C.c_int, [_CTX, C.c_uint32, _u8p]),
    "ske_hll_slab": (C.c_int, [_CTX, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "ske_hll_merge_groups_dev": (C.c_int, [_CTX, _u32p, _u32p, C.c_uint32, _u8p]),
    "ske_hll_count_raw_dev": (C.c_int, [_CTX, _u8p, C.c_uint32, _u64p]),
    "ske_swipes": (C.c_int, [_CTX, C.c_uint32, _u32p, _u8p, _u32p, C.c_uint64, _u8p, C.c_int]),
    "ske_swipes_async": (C.c_int, [_CTX, C.c_uint32, _u32p, _u8p, _u32p, C.c_uint64, _u8p]),
    "ske_swipes_fixed": (C.c_int, [_CTX, C.c_uint32, _u32p, _u8p, C.c_uint32, C.c_uint64, _u8p,
                                   C.c_int]),
    "ske_swipes_fixed_async": (C.c_int, [_CTX, C.c_uint32, _u32p, _u8p, C.c_uint32, C.c_uint64,
                                         _u8p]),
    "ske_swipes_many_async": (C.c_int, [_CTX, C.c_uint32, _vp, C.c_uint32, C.c_uint32]),
    "ske_swipes_fixed_bits": (C.c_int, [_CTX, C.c_uint32, _u32p, _u8p, C.c_uint32, C.c_uint64, _u8p, C.c_int]),
    "ske_route_swipes": (C.c_int, [_CTX, _u8p, C.c_uint32, _u32p, C.c_uint64, C.c_uint32, _u32p, _u32p,
                                   C.c_uint32, _u8p, _u32p, _u32p, _u64p]),
    "ske_route_swipes_cap_async": (C.c_int, [_CTX, _u8p, C.c_uint32, _u32p, C.c_uint64, C.c_uint32, _u32p,
                                             C.c_uint32, C.c_uint32, _u32p, _u8p, _u32p, _u32p, _u32p]),
    "ske_route_return_async": (C.c_int, [_CTX, _u8p, _u32p, C.c_uint64, _u8p]),
    "ske_route_slots_async": (C.c_int, [_CTX, _u32p, C.c_uint64, _u32p, C.c_uint32, C.c_uint32, _u32p]),
    "ske_swipes_stats": (C.c_int, [_CTX, C.c_uint32, _u8p, _u32p, C.c_uint64,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "ske_swipes_variant": (C.c_int, [_CTX, C.c_uint32]),
    "ske_set_option": (C.c_int, [_CTX, C.c_char_p, C.c_int64]),
    "ske_pass_times": (C.c_int, [_CTX, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]),
    "ske_ingest_parse": (C.c_int, [_CTX, _u8p, _u32p, C.c_uint64, C.c_int, C.POINTER(IngestCols)]),
    "ske_keytab_lookup": (C.c_int, [_CTX, C.POINTER(IngestCols), C.c_uint64, _u32p,
                                    C.POINTER(C.c_uint64)]),
    "ske_keytab_insert": (C.c_int, [_CTX, _u64p, _u32p, C.c_uint64]),
    "ske_keytab_clear": (C.c_int, [_CTX]),
    "ske_ingest_swipes": (C.c_int, [_CTX, C.c_uint32, _u8p, C.POINTER(IngestCols), C.c_uint64, _u8p,
                                    C.POINTER(C.c_uint64)]),
    "ske_capture_begin": (C.c_int, [_CTX]),
    "ske_capture_end": (C.c_int, [_CTX, C.POINTER(C.c_void_p)]),
    "ske_graph_launch": (C.c_int, [_CTX, _vp]),
    "ske_graph_free": (C.c_int, [_CTX, _vp]),
    "ske_gen_members": (C.c_int, [_CTX, C.POINTER(GenParams), C.c_uint64, C.c_uint64, _u8p, _u32p]),
    "ske_gen_swipes": (C.c_int, [_CTX, C.POINTER(GenParams), C.c_uint64, C.c_uint64, _u8p, _u32p,
                                 _u32p]),
    "ske_gen_id_width": (C.c_int, [C.POINTER(GenParams)]),
}

_lib = None


def load() -> C.CDLL:
    """Load libsketch.so and bind every symbol; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsketch.so is not built at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; "
            "g.build()'` (the sketch engine has no CPU fallback)")
    # One HIP runtime per process: libsketch and PyTorch-ROCm both need
    # libamdhip64.so.7 (same soname), and whichever loads first serves both.
    # PyTorch's runtime must be the one (its HIP stack fails to find the device
    # on top of /opt/rocm's), so torch is loaded before libsketch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("SKE_LIB") and not hasattr(lib, name):
            continue  # an A/B build of an older revision: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def strerror(code: int) -> str:
    return load().ske_strerror(code).decode()


def check(code: int, ctx=None) -> int:
    if code < 0:
        msg = strerror(code)
        if code in (SKE_EHIP, SKE_EBUSY) and ctx:
            msg += " (" + load().ske_last_hip_error(ctx).decode() + ")"
        raise SketchLibError(code, msg)
    return code


class Context:
    """One libsketch context (one HIP device, one stream)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        p = C.c_void_p()
        rc = self.lib.ske_open(device, C.byref(p))
        if rc != SKE_OK:
            raise SketchLibError(rc, f"ske_open(device={device}) failed: {strerror(rc)} -- "
                                     "a ROCm GPU is required (no CPU fallback)")
        self.ptr = p.value
        self.device = device

    def close(self):
        if getattr(self, "ptr", None):
            self.lib.ske_close(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def call(self, name: str, *args) -> int:
        return check(getattr(self.lib, name)(self.ptr, *args), self.ptr)
