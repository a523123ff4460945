"""ctypes binding of libhj.so (include/hj.h).

The HIP extension is the product: there is no CPU fallback.  If libhj.so is
missing this module raises at import time, loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("HJ_LIB", os.path.join(PKG_ROOT, "lib", "libhj.so"))
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "hj.h")

HJ_OK = 0
HJ_ERR_ARG = -1
HJ_ERR_HIP = -2
HJ_ERR_NOMEM = -3
HJ_ERR_STATE = -4
HJ_ERR_CAPACITY = -5

HJ_STRATEGY_AUTO = 0
HJ_STRATEGY_GLOBAL = 1
HJ_STRATEGY_RADIX = 2

_vp = C.c_void_p
_i64 = C.c_int64
_u64 = C.c_uint64
_int = C.c_int


def _load():
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so
    # (SONAME libamdhip64.so.7) and loads it by path.  Importing torch first
    # makes libhj.so's NEEDED libamdhip64.so.7 bind to that same instance
    # (matched by SONAME); loading libhj.so first would map /opt/rocm's copy
    # too, and two HSA runtimes in one process cannot share the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libhj.so not found at {LIB_PATH}: build it with `make -C mlir-hashjoin_amd` "
            "(or __graft_entry__.build()); the hash join has no CPU fallback")
    L = C.CDLL(LIB_PATH)
    sig = {
        "hj_abi_version": (_int, []),
        "hj_last_error": (C.c_char_p, []),
        "hj_device_info": (_int, [_int, C.POINTER(_i64)]),
        "hj_host_memo_hits": (_i64, []),
        "hj_host_set_reuse": (_int, [_int]),
        "hj_ctx_create": (_vp, [_int]),
        "hj_ctx_destroy": (None, [_vp]),
        "hj_ctx_reserve": (_int, [_vp, _i64, _int]),
        "hj_ctx_table_capacity": (_i64, [_vp]),
        "hj_ctx_radix_plan": (_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "hj_ctx_build_has_duplicates": (_int, [_vp]),
        "hj_ctx_join_kernel": (_int, [_vp]),
        "hj_ctx_set_timing": (_int, [_vp, _int]),
        "hj_ctx_last_timing": (_int, [_vp, C.POINTER(C.c_float)]),
        "hj_ctx_last_timing_ex": (_int, [_vp, C.POINTER(C.c_float)]),
        "hj_ctx_timing_accumulate": (_int, [_vp, _int]),
        "hj_ctx_timing_totals": (_int, [_vp, C.POINTER(C.c_float), C.POINTER(C.c_longlong)]),
        "hj_ctx_reserve_probe": (_int, [_vp, _i64, _int]),
        "hj_ctx_probe_hint": (_int, [_vp, _i64]),
        "hj_ctx_set_strategy": (_int, [_vp, _int]),
        "hj_ctx_strategy_used": (_int, [_vp]),
        "hj_ctx_set_radix_bits": (_int, [_vp, _int]),
        "hj_dev_build_i64": (_int, [_vp, _vp, _vp, _i64, _vp]),
        "hj_dev_count_i64": (_int, [_vp, _vp, _i64, _vp, _vp]),
        "hj_dev_probe_i64": (_int, [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_build_tuples_i64": (_int, [_vp, _vp, _i64, _vp]),
        "hj_dev_probe_tuples_i64": (_int, [_vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_build_i32": (_int, [_vp, _vp, _i64, _i64, _vp]),
        "hj_dev_count_i32": (_int, [_vp, _vp, _i64, _vp, _vp]),
        "hj_dev_probe_i32": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_partition_i64": (_int, [_vp, _vp, _vp, _i64, _int, _vp, _vp, _vp]),
        "hj_dev_partition_tuples_i64": (_int, [_vp, _vp, _i64, _int, _vp, _vp, _vp]),
        "hj_partition_of": (_int, [_i64, _int]),
        "hj_route_plan": (_int, [_i64, _int, C.POINTER(C.c_int)]),
        "hj_dev_route_i64": (_int, [_vp, _vp, _vp, _i64, _int, _int, _vp, _vp, _vp]),
        "hj_dev_build_routed_i64": (_int, [_vp, _vp, _i64, _vp, _int, _int, _int, _vp]),
        "hj_dev_probe_routed_i64": (_int, [_vp, _vp, _i64, _vp, _int, _int, _int, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_gen_pkfk_i64": (_int, [_u64, _i64, _u64, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp]),
        "hj_zipf_params": (_int, [_i64, C.c_double, C.POINTER(C.c_double)]),
        "hj_dev_gen_zipf_i64": (_int, [_u64, _i64, C.c_double, _i64, _i64, _vp, _vp, _vp]),
        "hj_dev_gen_uniform_i64": (_int, [_u64, _u64, _i64, _i64, _i64, _i64, _vp, _vp, _vp]),
        "hj_dev_gen_uniform_i32": (_int, [_u64, _u64, C.c_int32, C.c_int32, _i64, _i64, _vp, _vp]),
        "hj_count_i32": (_i64, [_vp, _vp, _i64, _i64, _i64] * 2),
        "hj_probe_i32": (C.c_int32, [_vp, _vp, _i64, _i64, _i64] * 4),
        "hj_count_i64": (_i64, [_vp, _vp, _i64, _i64, _i64] * 4),
        "hj_probe_i64": (C.c_int32, [_vp, _vp, _i64, _i64, _i64] * 6),
        "hj_dev_count_rows_i32": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _vp]),
        "hj_dev_join_rows_i32": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp,
                                        _vp]),
        "hj_count_rows_i32": (_i64, [_vp, _vp, _i64, _i64, _i64, _i64, _i64] * 2),
        "hj_join_rows_i32": (_i64, [_vp, _vp, _i64, _i64, _i64, _i64, _i64] * 3),
        "_mlir_ciface_hj_join_rows_i32": (None, [_vp, _vp, _vp]),
        "hj_host_join_ooc_i64": (_i64, [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _u64]),
        "hj_dev_select_f32": (_int, [_vp, _vp, _i64, _int, C.c_float, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_select_i64": (_int, [_vp, _vp, _i64, _int, _i64, _vp, _vp, _i64, _vp, _vp]),
        "hj_dev_stream_copy": (_int, [_vp, _vp, _i64, _int, _vp]),
        "hj_placement_stats": (None, [_vp, _vp, _vp, _vp]),
        "hj_placement_stats_ex": (None, [_vp, _vp, _vp]),
        "hj_placement_set_good": (C.c_double, [C.c_double]),
        "hj_placement_check": (_int, [_vp, _i64, _vp]),
        "hj_select_f32": (_i64, [_vp, _vp, _i64, _i64, _i64, C.c_float, _vp, _vp, _i64, _i64, _i64]),
        "_mlir_ciface_hj_join_i32": (None, [_vp, _vp, _vp]),
        "_mlir_ciface_hj_join_i64": (None, [_vp, _vp, _vp]),
        "_mlir_ciface_hj_join_kp_i64": (None, [_vp, _vp, _vp, _vp, _vp]),
        "hj_free_result": (None, [_vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


class HJError(RuntimeError):
    pass


def check(rc, what=""):
    if rc != HJ_OK:
        msg = lib.hj_last_error().decode(errors="replace")
        raise HJError(f"{what} failed with {rc}: {msg}")
    return rc


def declared_symbols():
    """Every function name include/hj.h declares (for the ABI export test)."""
    import re
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", text, flags=re.M)
    return sorted({n for n in names if n.startswith(("hj_", "_mlir_ciface_hj_"))})


def memref_struct(ctype, rank):
    class _M(C.Structure):
        _fields_ = [("allocated", C.POINTER(ctype)), ("aligned", C.POINTER(ctype)), ("offset", _i64),
                    ("sizes", _i64 * rank), ("strides", _i64 * rank)]
    return _M


MemRef1I32 = memref_struct(C.c_int32, 1)
MemRef1I64 = memref_struct(C.c_int64, 1)
MemRef2I32 = memref_struct(C.c_int32, 2)
MemRef2I64 = memref_struct(C.c_int64, 2)
