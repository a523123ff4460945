"""The host memref ABI of libhj.so called the way lowered MLIR calls it.

A ranked memref<?xT> argument becomes five scalars (allocated, aligned,
offset, size, stride) after -finalize-memref-to-llvm (join_v1.ll:1262-1265);
`expand()` produces exactly that tuple from a numpy array view, including
non-zero offsets and non-unit strides.  The C-interface forms take
descriptor pointers (result first).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MemRef1I32, MemRef1I64, MemRef2I32, MemRef2I64, check, lib

_CT = {np.dtype(np.int32): C.c_int32, np.dtype(np.int64): C.c_int64}


def expand(a: np.ndarray, base: np.ndarray | None = None):
    """5-scalar expansion of a 1-D view `a` of `base` (allocated/aligned =
    base pointer, offset/stride in elements)."""
    base = a if base is None else base
    item = a.itemsize
    if a.ndim != 1 or a.strides[0] % item:
        raise ValueError("1-D element-strided view required")
    ptr = base.ctypes.data
    off = (a.ctypes.data - ptr) // item
    stride = a.strides[0] // item if a.shape[0] > 1 else 1
    return [C.c_void_p(ptr), C.c_void_p(ptr), off, a.shape[0], stride]


def count_i32(r, s, r_base=None, s_base=None):
    """@countRows through hj_count_i32 (returns M, or a negative error)."""
    return int(lib.hj_count_i32(*expand(r, r_base), *expand(s, s_base)))


def probe_i32(r, s, out_r, out_s):
    return int(lib.hj_probe_i32(*expand(r), *expand(s), *expand(out_r), *expand(out_s)))


def count_i64(rk, rp, sk, sp):
    return int(lib.hj_count_i64(*expand(rk), *expand(rp), *expand(sk), *expand(sp)))


def probe_i64(rk, rp, sk, sp, out_r, out_s):
    return int(lib.hj_probe_i64(*expand(rk), *expand(rp), *expand(sk), *expand(sp), *expand(out_r),
                                *expand(out_s)))


def join_i32_two_phase(r, s):
    """count -> allocate -> probe, the reference @main order (join_v2.mlir:672-696)."""
    m = count_i32(r, s)
    if m < 0:
        check(m, "hj_count_i32")
    out_r = np.empty(m, np.int32); out_s = np.empty(m, np.int32)
    check(probe_i32(r, s, out_r, out_s), "hj_probe_i32")
    return out_r, out_s


def expand2(a: np.ndarray, base: np.ndarray | None = None):
    """7-scalar expansion of a 2-D memref<?x?xT> view (allocated, aligned,
    offset, sizes[2], strides[2], all in elements)."""
    base = a if base is None else base
    item = a.itemsize
    if a.ndim != 2 or a.strides[0] % item or a.strides[1] % item:
        raise ValueError("2-D element-strided view required")
    ptr = base.ctypes.data
    off = (a.ctypes.data - ptr) // item
    return [C.c_void_p(ptr), C.c_void_p(ptr), off, a.shape[0], a.shape[1], a.strides[0] // item,
            a.strides[1] // item]


def count_rows_i32(t1, t2):
    """nested-loop.mlir result row count through hj_count_rows_i32."""
    return int(lib.hj_count_rows_i32(*expand2(t1), *expand2(t2)))


def join_rows_i32(t1, t2, out):
    """nested-loop.mlir rows into the 2-D result memref `out`; returns M."""
    return int(lib.hj_join_rows_i32(*expand2(t1), *expand2(t2), *expand2(out)))


def ciface_join_rows_i32(t1, t2):
    """_mlir_ciface_hj_join_rows_i32: memref<?x?xi32> x2 -> memref<?x?xi32> rows."""
    t1 = np.ascontiguousarray(t1, np.int32); t2 = np.ascontiguousarray(t2, np.int32)
    res = MemRef2I32()
    ds = []
    for t in (t1, t2):
        d = MemRef2I32()
        p = t.ctypes.data_as(C.POINTER(C.c_int32))
        d.allocated = p; d.aligned = p; d.offset = 0
        d.sizes[0], d.sizes[1] = t.shape
        d.strides[0], d.strides[1] = t.shape[1], 1
        ds.append(d)
    lib._mlir_ciface_hj_join_rows_i32(C.byref(res), C.byref(ds[0]), C.byref(ds[1]))
    if not res.allocated:
        raise RuntimeError("ciface join failed: " + lib.hj_last_error().decode())
    m, oc = res.sizes[0], res.sizes[1]
    out = np.ctypeslib.as_array(res.aligned, shape=(max(m * oc, 1),))[: m * oc].reshape(m, oc).copy()
    lib.hj_free_result(C.cast(res.allocated, C.c_void_p))
    return out


def select_f32(a, value, out, a_base=None, out_base=None):
    """selection.mlir over host memrefs: a[i] < value compacted into `out`; returns M."""
    return int(lib.hj_select_f32(*expand(a, a_base), C.c_float(value), *expand(out, out_base)))


def _desc1(a, cls):
    d = cls()
    ct = _CT[a.dtype]
    p = a.ctypes.data_as(C.POINTER(ct))
    d.allocated = p
    d.aligned = p
    d.offset = 0
    d.sizes[0] = a.shape[0]
    d.strides[0] = a.strides[0] // a.itemsize if a.shape[0] > 1 else 1
    return d


def _take_result(res, dtype):
    m = res.sizes[0]
    if m < 0:
        raise RuntimeError("ciface join failed: " + lib.hj_last_error().decode())
    out = np.ctypeslib.as_array(res.aligned, shape=(max(m, 1) * 2,))[: m * 2].reshape(m, 2).astype(dtype, copy=True)
    lib.hj_free_result(C.cast(res.allocated, C.c_void_p))
    return out


def ciface_join_i32(r, s):
    """_mlir_ciface_hj_join_i32: memref<?xi32> x2 -> memref<?x2xi32>."""
    r = np.ascontiguousarray(r, np.int32); s = np.ascontiguousarray(s, np.int32)
    res = MemRef2I32()
    dr, ds = _desc1(r, MemRef1I32), _desc1(s, MemRef1I32)
    lib._mlir_ciface_hj_join_i32(C.byref(res), C.byref(dr), C.byref(ds))
    if not res.allocated:
        raise RuntimeError("ciface join failed: " + lib.hj_last_error().decode())
    return _take_result(res, np.int32)


def ciface_join_i64(r, s):
    r = np.ascontiguousarray(r, np.int64); s = np.ascontiguousarray(s, np.int64)
    res = MemRef2I64()
    dr, ds = _desc1(r, MemRef1I64), _desc1(s, MemRef1I64)
    lib._mlir_ciface_hj_join_i64(C.byref(res), C.byref(dr), C.byref(ds))
    if not res.allocated:
        raise RuntimeError("ciface join failed: " + lib.hj_last_error().decode())
    return _take_result(res, np.int64)


def ciface_join_kp_i64(rk, rp, sk, sp):
    arrs = [np.ascontiguousarray(a, np.int64) for a in (rk, rp, sk, sp)]
    res = MemRef2I64()
    ds = [_desc1(a, MemRef1I64) for a in arrs]
    lib._mlir_ciface_hj_join_kp_i64(C.byref(res), *[C.byref(d) for d in ds])
    if not res.allocated:
        raise RuntimeError("ciface join failed: " + lib.hj_last_error().decode())
    return _take_result(res, np.int64)
