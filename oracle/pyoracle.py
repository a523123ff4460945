"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU oracle (hj_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline.  The product path
(mlir-hashjoin_amd/) never imports it.

Also exposes the reference's own ``check()`` (shared_stuff/shared.cpp:129-172)
compiled into oracle/_ref/shared.so, called through the expanded memref ABI
exactly as the lowered join_v1.ll:1228 does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "shared.so")

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u64 = C.c_uint64
_i64 = C.c_int64

_lib = None
_ref = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_fmix64.restype = _u64
        L.oracle_fmix64.argtypes = [_u64]
        L.oracle_rand.restype = _u64
        L.oracle_rand.argtypes = [_u64, _u64, _u64]
        L.oracle_gen_pkfk_i64.restype = None
        L.oracle_gen_pkfk_i64.argtypes = [_u64, _i64, _u64, _i64, _i64, _i64p, _i64p, _i64, _i64, _i64p, _i64p]
        L.oracle_gen_zipf_i64.restype = None
        L.oracle_gen_zipf_i64.argtypes = [_u64, _i64, C.c_double, C.c_double, C.c_double, C.c_double, _i64, _i64,
                                          _i64p, _i64p]
        L.oracle_gen_uniform_i64.restype = None
        L.oracle_gen_uniform_i64.argtypes = [_u64, _u64, _i64, _i64, _i64, _i64, _i64p, _i64p]
        L.oracle_gen_uniform_i32.restype = None
        L.oracle_gen_uniform_i32.argtypes = [_u64, _u64, C.c_int32, C.c_int32, _i64, _i64, _i32p]
        L.oracle_chained_join_i64.restype = _i64
        L.oracle_chained_join_i64.argtypes = [C.c_void_p, C.c_void_p, _i64, C.c_void_p, C.c_void_p, _i64,
                                              _u64, C.c_int, C.c_void_p, C.c_void_p, _i64]
        L.oracle_chained_join_i32.restype = _i64
        L.oracle_chained_join_i32.argtypes = [C.c_void_p, _i64, C.c_void_p, _i64, C.c_uint32, C.c_int,
                                              C.c_void_p, C.c_void_p, _i64]
        L.oracle_chained_join_i64_omp.restype = _i64
        L.oracle_chained_join_i64_omp.argtypes = [C.c_void_p, C.c_void_p, _i64, C.c_void_p, C.c_void_p, _i64,
                                                  _u64, C.c_int, C.c_void_p, C.c_void_p, _i64, C.c_void_p]
        L.oracle_nested_loop_i64.restype = _i64
        L.oracle_nested_loop_i64.argtypes = [C.c_void_p, C.c_void_p, _i64, C.c_void_p, C.c_void_p, _i64,
                                             C.c_void_p, C.c_void_p, _i64]
        L.oracle_nested_loop_i32.restype = _i64
        L.oracle_nested_loop_i32.argtypes = [C.c_void_p, _i64, C.c_void_p, _i64, C.c_void_p, C.c_void_p, _i64]
        L.oracle_nested_loop_count_i64_omp.restype = _i64
        L.oracle_nested_loop_count_i64_omp.argtypes = [C.c_void_p, _i64, C.c_void_p, _i64, C.c_int]
        L.oracle_nested_join_rows_i32.restype = _i64
        L.oracle_nested_join_rows_i32.argtypes = [C.c_void_p, _i64, _i64, C.c_void_p, _i64, _i64, C.c_void_p, _i64]
        L.oracle_nested_init_i32.restype = None
        L.oracle_nested_init_i32.argtypes = [C.c_void_p, _i64, _i64]
        L.oracle_select_f32.restype = _i64
        L.oracle_select_f32.argtypes = [C.c_void_p, _i64, C.c_int, C.c_float, C.c_void_p, C.c_void_p, _i64]
        L.oracle_select_i64.restype = _i64
        L.oracle_select_i64.argtypes = [C.c_void_p, _i64, C.c_int, _i64, C.c_void_p, C.c_void_p, _i64]
        L.oracle_selection_init_f32.restype = None
        L.oracle_selection_init_f32.argtypes = [C.c_void_p, _i64]
        L.oracle_pair_digest_i64.restype = None
        L.oracle_pair_digest_i64.argtypes = [C.c_void_p, C.c_void_p, _i64, C.POINTER(_u64), C.POINTER(_u64)]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


U64_MAX = (1 << 64) - 1


def hit_threshold(frac: float) -> int:
    """Match-fraction knob of the PK-FK generator as a uint64 threshold."""
    if frac >= 1.0:
        return U64_MAX
    return min(U64_MAX - 1, int(frac * float(1 << 64)))


# ---------------------------------------------------------------- generators
def gen_pkfk_i64(seed, NR, NS, frac=1.0, r0=0, nr=None, s0=0, ns=None):
    nr = NR if nr is None else nr
    ns = NS if ns is None else ns
    rk = np.empty(nr, np.int64); rp = np.empty(nr, np.int64)
    sk = np.empty(ns, np.int64); sp = np.empty(ns, np.int64)
    lib().oracle_gen_pkfk_i64(seed, NR, hit_threshold(frac), r0, nr, rk, rp, s0, ns, sk, sp)
    return rk, rp, sk, sp


def gen_zipf_i64(seed, NR, params, s0=0, ns=0):
    """params = hashjoin.zipf_params(NR, theta) (zeta, eta, alpha, 0.5^theta)."""
    sk = np.empty(ns, np.int64); sp = np.empty(ns, np.int64)
    lib().oracle_gen_zipf_i64(seed, NR, params[0], params[1], params[2], params[3], s0, ns, sk, sp)
    return sk, sp


def gen_uniform_i64(seed, stream, lo, hi, n, i0=0):
    k = np.empty(n, np.int64); p = np.empty(n, np.int64)
    lib().oracle_gen_uniform_i64(seed, stream, lo, hi, i0, n, k, p)
    return k, p


def gen_uniform_i32(seed, stream, lo, hi, n, i0=0):
    k = np.empty(n, np.int32)
    lib().oracle_gen_uniform_i32(seed, stream, lo, hi, i0, n, k)
    return k


def pkfk_expected(seed, NR, NS, frac=1.0, s0=0, ns=None):
    """(r_pay, s_pay) pairs the PK-FK generator promises, computed from the
    generator's definition (independent of any join)."""
    ns = NS if ns is None else ns
    L = lib()
    thr = hit_threshold(frac)
    rs, ss = [], []
    for j in range(ns):
        g = s0 + j
        u = L.oracle_rand(seed, 1, g) % NR
        if thr == U64_MAX or L.oracle_rand(seed, 2, g) < thr:
            rs.append(u); ss.append(g)
    return np.array(rs, np.int64), np.array(ss, np.int64)


# ---------------------------------------------------------------- joins
def chained_join_i64(rk, rp, sk, sp, H=None, variant=2, count_only=False):
    """join_v1/v2 restated (variant 1/2).  Returns (out_r, out_s) or M."""
    L = lib()
    rk = np.ascontiguousarray(rk, np.int64); sk = np.ascontiguousarray(sk, np.int64)
    rp = None if rp is None else np.ascontiguousarray(rp, np.int64)
    sp = None if sp is None else np.ascontiguousarray(sp, np.int64)
    H = max(1, len(rk)) if H is None else H
    m = L.oracle_chained_join_i64(_p(rk), _p(rp), len(rk), _p(sk), _p(sp), len(sk), H, variant, None, None, 0)
    if m < 0:
        raise MemoryError("oracle allocation failed")
    if count_only:
        return m
    o_r = np.empty(max(m, 1), np.int64); o_s = np.empty(max(m, 1), np.int64)
    m2 = L.oracle_chained_join_i64(_p(rk), _p(rp), len(rk), _p(sk), _p(sp), len(sk), H, variant, _p(o_r), _p(o_s), m)
    assert m2 == m
    return o_r[:m], o_s[:m]


def chained_join_i32(r, s, H=None, variant=2):
    L = lib()
    r = np.ascontiguousarray(r, np.int32); s = np.ascontiguousarray(s, np.int32)
    H = max(1, len(r)) if H is None else H
    m = L.oracle_chained_join_i32(_p(r), len(r), _p(s), len(s), H, variant, None, None, 0)
    o_r = np.empty(max(m, 1), np.int32); o_s = np.empty(max(m, 1), np.int32)
    L.oracle_chained_join_i32(_p(r), len(r), _p(s), len(s), H, variant, _p(o_r), _p(o_s), m)
    return o_r[:m], o_s[:m]


def chained_join_i64_omp(rk, rp, sk, sp, H, threads, count_only=False):
    """Host-thread grid of join_v2 (CPU baseline).  Returns (M, phase_seconds[4])."""
    L = lib()
    ph = np.zeros(4, np.float64)
    if count_only:
        o_r = o_s = None; cap = 0
    else:
        cap = len(sk) * 2 + 16
        o_r = np.empty(cap, np.int64); o_s = np.empty(cap, np.int64)
    m = L.oracle_chained_join_i64_omp(_p(rk), _p(rp), len(rk), _p(sk), _p(sp), len(sk), H, threads,
                                      _p(o_r), _p(o_s), cap, _p(ph))
    return m, ph


def nested_loop_i64(rk, rp, sk, sp):
    L = lib()
    m = L.oracle_nested_loop_i64(_p(rk), _p(rp), len(rk), _p(sk), _p(sp), len(sk), None, None, 0)
    o_r = np.empty(max(m, 1), np.int64); o_s = np.empty(max(m, 1), np.int64)
    L.oracle_nested_loop_i64(_p(rk), _p(rp), len(rk), _p(sk), _p(sp), len(sk), _p(o_r), _p(o_s), m)
    return o_r[:m], o_s[:m]


def nested_loop_i32(r, s):
    L = lib()
    r = np.ascontiguousarray(r, np.int32); s = np.ascontiguousarray(s, np.int32)
    m = L.oracle_nested_loop_i32(_p(r), len(r), _p(s), len(s), None, None, 0)
    o_r = np.empty(max(m, 1), np.int32); o_s = np.empty(max(m, 1), np.int32)
    L.oracle_nested_loop_i32(_p(r), len(r), _p(s), len(s), _p(o_r), _p(o_s), m)
    return o_r[:m], o_s[:m]


def nested_join_rows_i32(t1, t2):
    L = lib()
    t1 = np.ascontiguousarray(t1, np.int32); t2 = np.ascontiguousarray(t2, np.int32)
    (r1, c1), (r2, c2) = t1.shape, t2.shape
    oc = c1 + c2 - 1
    m = L.oracle_nested_join_rows_i32(_p(t1), r1, c1, _p(t2), r2, c2, None, 0)
    out = np.zeros((max(m, 1), oc), np.int32)
    L.oracle_nested_join_rows_i32(_p(t1), r1, c1, _p(t2), r2, c2, _p(out), m)
    return out[:m]


def nested_init_i32(rows, cols):
    t = np.empty((rows, cols), np.int32)
    lib().oracle_nested_init_i32(_p(t), rows, cols)
    return t


CMP = {"lt": 0, "le": 1, "gt": 2, "ge": 3, "eq": 4, "ne": 5}


def select(a, op, c):
    """selection.mlir restated: (values, row indices) of a[i] <op> c, in order."""
    L = lib()
    if a.dtype == np.float32:
        a = np.ascontiguousarray(a); f = L.oracle_select_f32; c = float(c)
    else:
        a = np.ascontiguousarray(a, np.int64); f = L.oracle_select_i64; c = int(c)
    m = f(_p(a), len(a), CMP[op], c, None, None, 0)
    out = np.empty(max(m, 1), a.dtype); rows = np.empty(max(m, 1), np.int64)
    f(_p(a), len(a), CMP[op], c, _p(out), _p(rows), m)
    return out[:m], rows[:m]


def selection_init_f32(n):
    a = np.empty(n, np.float32)
    lib().oracle_selection_init_f32(_p(a), n)
    return a


def pair_digest(r, s):
    r = np.ascontiguousarray(r, np.int64); s = np.ascontiguousarray(s, np.int64)
    a = _u64(0); b = _u64(0)
    lib().oracle_pair_digest_i64(_p(r), _p(s), len(r), C.byref(a), C.byref(b))
    return a.value, b.value


def sorted_pairs(r, s):
    """Lexicographically sorted (r, s) pairs as an (M, 2) int64 array --
    the comparison shared.cpp:168-171 performs."""
    r = np.asarray(r, np.int64); s = np.asarray(s, np.int64)
    order = np.lexsort((s, r))
    return np.stack([r[order], s[order]], axis=1)


def same_multiset(r1, s1, r2, s2):
    """Exact row count, then sorted compare (check() alone has a
    false positive on extra (0,0) rows, so the count is compared first)."""
    if len(r1) != len(r2) or len(s1) != len(s2) or len(r1) != len(s1):
        return False
    return bool(np.array_equal(sorted_pairs(r1, s1), sorted_pairs(r2, s2)))


# ---------------------------------------------------------------- reference
def ref_available():
    return os.path.exists(REF_PATH)


def ref_check(r, s, out_r, out_s):
    """Call the reference's own check() (shared.cpp:129-172) through the
    expanded 5-argument memref ABI (join_v1.ll:1228).  1 / 0 / -1."""
    global _ref
    if _ref is None:
        _ref = C.CDLL(REF_PATH)
        mr = [C.c_void_p, C.c_void_p, _i64, _i64, _i64]
        _ref.check.restype = C.c_int32
        _ref.check.argtypes = mr * 4
    arrs = [np.ascontiguousarray(a, np.int32) for a in (r, s, out_r, out_s)]
    args = []
    for a in arrs:
        p = a.ctypes.data_as(C.c_void_p)
        args += [p, p, 0, len(a), 1]
    return int(_ref.check(*args))
