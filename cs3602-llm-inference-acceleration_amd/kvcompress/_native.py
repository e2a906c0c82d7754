"""ctypes binding of libkvc.so (include/kvc.h).

The HIP library is the only compute path of this package: if it is missing or cannot be
loaded, every compressing call raises -- there is no CPU or eager-PyTorch fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libkvc.so")
# diagnostic builds (e.g. the s_memtime-stamped select kernel) may be swapped in by path
LIB_PATH = os.environ.get("KVC_LIB", LIB_PATH)

KVC_F32, KVC_BF16, KVC_F16 = 0, 1, 2
KVC_ASC, KVC_DESC = 0, 1
KVC_ALGO_SORT, KVC_ALGO_TOPK, KVC_ALGO_STABLE = 0, 1, 2
KVC_SCORE_NORM, KVC_SCORE_SNAPKV = 0, 1
PHASE_SCORE, PHASE_SELECT, PHASE_GATHER, PHASE_ALL = 1, 2, 4, 7
FLAG_SPLIT_SELECT_GATHER, FLAG_SHARED_INDEX, FLAG_GATHER_FIXED, FLAG_GATHER_SELECTED = 1, 2, 4, 8
DEV_SELECT_BOUNDS, DEV_INDEX_RANGE, DEV_INTERNAL = 1, 2, 4  # enum kvc_device_status bits


ATTN_HH_STABLE = 4  # kvc_attn_params.flags: kvc_heavy_hitters with the stable tie order


def ATTN_OLD_DTYPE(d):
    """kvc_attn_params.flags of kvc_attn_accumulate: acc_old of dtype d (KVC_ATTN_OLD_DTYPE)."""
    return d + 1

ABI_VERSION = 4
KVC_E_TOO_LONG = -5

# struct kvc_layer (include/kvc.h) -- 136 bytes, checked against kvc_layer_struct_size()
LAYER_DTYPE = np.dtype([
    ("k", "<u8"), ("v", "<u8"), ("k_out", "<u8"), ("v_out", "<u8"),
    ("k_stride", "<i8", (3,)), ("v_stride", "<i8", (3,)),
    ("seq_len", "<i4"), ("zone_start", "<i4"), ("zone_len", "<i4"), ("n_select", "<i4"),
    ("sink_len", "<i4"), ("tail_start", "<i4"), ("tail_len", "<i4"), ("pool_kernel", "<i4"),
    ("score_mode", "<i4"), ("n_out", "<i4"), ("row0", "<i4"), ("tile0", "<i4"),
    ("unit0", "<i8"),
])
assert LAYER_DTYPE.itemsize == 136

# struct kvc_attn_layer / kvc_hh_layer (include/kvc.h: h2o_attention heavy hitters)
ATTN_LAYER_DTYPE = np.dtype([
    ("attn", "<u8"), ("attn_stride", "<i8", (3,)), ("acc_old", "<u8"), ("acc_new", "<u8"),
    ("q_len", "<i4"), ("key_len", "<i4"), ("old_len", "<i4"), ("col_chunk", "<i4"),
])
assert ATTN_LAYER_DTYPE.itemsize == 64
HH_LAYER_DTYPE = np.dtype([
    ("acc", "<u8"), ("acc_len", "<i4"), ("zone_start", "<i4"), ("zone_len", "<i4"),
    ("n_select", "<i4"), ("col_chunk", "<i4"), ("reserved", "<i4"),
])
assert HH_LAYER_DTYPE.itemsize == 32


class Params(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("batch", ctypes.c_int32), ("heads", ctypes.c_int32),
                ("head_dim", ctypes.c_int32), ("order", ctypes.c_int32), ("algo", ctypes.c_int32),
                ("phases", ctypes.c_int32), ("external_index", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("device_status", ctypes.c_void_p)]


class AttnParams(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("batch", ctypes.c_int32), ("heads", ctypes.c_int32),
                ("vec_bytes", ctypes.c_int32), ("decay", ctypes.c_float),
                ("flags", ctypes.c_int32), ("device_status", ctypes.c_void_p)]


class PlanInfo(ctypes.Structure):
    _fields_ = [("norm_offset", ctypes.c_size_t),
                ("index_offset", ctypes.c_size_t), ("workspace_bytes", ctypes.c_size_t),
                ("norm_row_stride", ctypes.c_int64), ("index_row_stride", ctypes.c_int64),
                ("rows", ctypes.c_int64), ("score_tiles", ctypes.c_int64),
                ("gather_units", ctypes.c_int64)]


EXPORTS = ("kvc_version", "kvc_layer_struct_size", "kvc_max_zone_len", "kvc_status_string",
           "kvc_source_digest",
           "kvc_plan", "kvc_launch", "kvc_compress", "kvc_attn_accumulate", "kvc_hh_workspace",
           "kvc_heavy_hitters", "kvc_debug_select_capacity")

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def lib():
    """Load libkvc.so once; raise loudly if it is absent or incompatible."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"HIP engine library not built: {LIB_PATH} is missing. "
            "Build it with `python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950).")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.kvc_version.restype = i32
    L.kvc_layer_struct_size.restype = ctypes.c_size_t
    L.kvc_max_zone_len.restype = i32
    L.kvc_status_string.restype = ctypes.c_char_p
    L.kvc_status_string.argtypes = [i32]
    L.kvc_source_digest.restype = ctypes.c_char_p
    L.kvc_source_digest.argtypes = []
    L.kvc_plan.restype = i32
    L.kvc_plan.argtypes = [ctypes.POINTER(Params), vp, i32, ctypes.POINTER(PlanInfo)]
    L.kvc_launch.restype = i32
    L.kvc_launch.argtypes = [ctypes.POINTER(Params), vp, i32, vp, ctypes.c_size_t, vp]
    L.kvc_compress.restype = i32
    L.kvc_compress.argtypes = [ctypes.POINTER(Params), vp, i32, vp, ctypes.c_size_t, vp]
    L.kvc_attn_accumulate.restype = i32
    L.kvc_attn_accumulate.argtypes = [ctypes.POINTER(AttnParams), vp, i32, vp]
    L.kvc_hh_workspace.restype = i32
    L.kvc_hh_workspace.argtypes = [ctypes.POINTER(AttnParams), vp, i32,
                                   ctypes.POINTER(ctypes.c_size_t)]
    L.kvc_heavy_hitters.restype = i32
    L.kvc_heavy_hitters.argtypes = [ctypes.POINTER(AttnParams), vp, i32, vp, ctypes.c_int64, vp,
                                    ctypes.c_size_t, vp]
    L.kvc_debug_select_capacity.restype = i32
    L.kvc_debug_select_capacity.argtypes = [ctypes.POINTER(Params), vp, i32, vp, ctypes.c_size_t,
                                            i32, vp]
    if L.kvc_version() != ABI_VERSION or L.kvc_layer_struct_size() != LAYER_DTYPE.itemsize:
        raise NativeLibraryError("libkvc.so ABI mismatch; rebuild it")
    _lib = L
    return L


def source_digest():
    """SHA-256 of the sources libkvc.so was built from ("unknown" for variant builds)."""
    return lib().kvc_source_digest().decode()


def status_string(rc):
    return lib().kvc_status_string(rc).decode()


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {status_string(rc)} (kvc status {rc})")


def plan(params, table):
    info = PlanInfo()
    rc = lib().kvc_plan(ctypes.byref(params), table.ctypes.data, len(table), ctypes.byref(info))
    return rc, info


def launch(params, table, ws_ptr, ws_bytes, stream_ptr):
    return lib().kvc_launch(ctypes.byref(params), table.ctypes.data, len(table), ws_ptr, ws_bytes,
                            stream_ptr)


def attn_accumulate(params, table, stream_ptr):
    return lib().kvc_attn_accumulate(ctypes.byref(params), table.ctypes.data, len(table),
                                     stream_ptr)


def hh_workspace(params, table):
    n = ctypes.c_size_t()
    rc = lib().kvc_hh_workspace(ctypes.byref(params), table.ctypes.data, len(table),
                                ctypes.byref(n))
    return rc, n.value


def heavy_hitters(params, table, out_ptr, out_stride, ws_ptr, ws_bytes, stream_ptr):
    return lib().kvc_heavy_hitters(ctypes.byref(params), table.ctypes.data, len(table), out_ptr,
                                   out_stride, ws_ptr, ws_bytes, stream_ptr)


def debug_select_capacity(params, table, ws_ptr, ws_bytes, zone_cap, stream_ptr):
    """kvc_debug_select_capacity: the test hook of the device-side selection bounds check."""
    return lib().kvc_debug_select_capacity(ctypes.byref(params), table.ctypes.data, len(table),
                                           ws_ptr, ws_bytes, zone_cap, stream_ptr)
