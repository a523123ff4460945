"""Host-side mirror of the reference's join program over device tensors.

The reference's host functions (join_v2.mlir:25-199) map one-to-one:

    @allocateHashTable     -> HashJoin.allocate_hash_table   (hj_ctx_reserve)
    @initializeHashTable   -> HashJoin.build_table           (init + build
    @buildTable               kernels, hj_dev_build_*)
    @countRows             -> HashJoin.count_rows            (hj_dev_count_*)
    @probeRelation         -> HashJoin.probe_relation        (hj_dev_probe_*)
    @main's join sequence  -> HashJoin.join

Tensors are PyTorch device tensors (plumbing only: allocation and the HIP
stream); every computation runs in libhj.so's HIP kernels.  Key dtype picks
the table layout: int64 keys -> 64-bit key/payload columns, int32 keys -> the
reference's i32 keys with i32 row ids.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from ._lib import HJ_STRATEGY_AUTO, HJ_STRATEGY_GLOBAL, HJ_STRATEGY_RADIX, check, lib

STRATEGIES = {"auto": HJ_STRATEGY_AUTO, "global": HJ_STRATEGY_GLOBAL, "radix": HJ_STRATEGY_RADIX}


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device, stream=None):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return C.c_void_p(s.cuda_stream)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("hash join inputs must be contiguous device tensors")


class HashJoin:
    """One device's hash-join context (table workspace + phase timing)."""

    def __init__(self, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("HashJoin needs a HIP device (no CPU fallback)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._ctx = lib.hj_ctx_create(self.device.index)
        if not self._ctx:
            raise RuntimeError("hj_ctx_create failed: " + lib.hj_last_error().decode())
        self._count = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.key_bits = None
        self._routed = {}   # slot -> (rows, 2) int64 routed-tuple buffer (route(..., slot=))

    def close(self):
        self._routed = {}
        if getattr(self, "_ctx", None):
            lib.hj_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- workspace
    def allocate_hash_table(self, num_tuples, key_bits=64):
        """@allocateHashTable (join_v2.mlir:25-39): size the workspace once."""
        check(lib.hj_ctx_reserve(self._ctx, int(num_tuples), int(key_bits)), "hj_ctx_reserve")

    def reserve_probe(self, num_tuples, key_bits=64):
        check(lib.hj_ctx_reserve_probe(self._ctx, int(num_tuples), int(key_bits)), "hj_ctx_reserve_probe")

    def probe_hint(self, num_tuples):
        """The probe side's expected rows, given before the build (None or < 0:
        unknown).  AUTO spares a mid-size build the radix partition it keeps
        only for probe sides of >= 2^24 rows (hj_ctx_probe_hint)."""
        check(lib.hj_ctx_probe_hint(self._ctx, -1 if num_tuples is None else int(num_tuples)), "hj_ctx_probe_hint")

    def set_strategy(self, name, radix_bits=0):
        """'auto' | 'global' (one HBM table) | 'radix' (partitioned, LDS tables);
        radix_bits > 0 fixes the partition count to 2^radix_bits."""
        check(lib.hj_ctx_set_strategy(self._ctx, STRATEGIES[name]), "hj_ctx_set_strategy")
        check(lib.hj_ctx_set_radix_bits(self._ctx, int(radix_bits)), "hj_ctx_set_radix_bits")

    @property
    def strategy_used(self):
        return {HJ_STRATEGY_GLOBAL: "global", HJ_STRATEGY_RADIX: "radix"}.get(
            lib.hj_ctx_strategy_used(self._ctx), None)

    @property
    def capacity(self):
        return int(lib.hj_ctx_table_capacity(self._ctx))

    @property
    def radix_plan(self):
        """Fan-out bits per partition pass of the current radix build ([] for global)."""
        n = C.c_int(0)
        bits = (C.c_int * 3)()
        check(lib.hj_ctx_radix_plan(self._ctx, C.byref(n), bits), "hj_ctx_radix_plan")
        return [bits[i] for i in range(n.value)]

    @property
    def radix_passes(self):
        return len(self.radix_plan)

    def has_duplicates(self):
        r = lib.hj_ctx_build_has_duplicates(self._ctx)
        if r < 0:
            check(r, "hj_ctx_build_has_duplicates")
        return bool(r)

    JOIN_KERNELS = {1: "k_join_b", 2: "k_join_u", 3: "k_join_u_stream", 4: "k_join_grp", 5: "k_join"}

    @property
    def join_kernel(self):
        """Kernel of the last radix join (hj_ctx_join_kernel): 'k_join_b',
        'k_join_u_stream', 'k_join_grp', 'k_join', or None (no radix join)."""
        r = lib.hj_ctx_join_kernel(self._ctx)
        if r < 0:
            check(r, "hj_ctx_join_kernel")
        return self.JOIN_KERNELS.get(r)

    def set_timing(self, enable=True):
        check(lib.hj_ctx_set_timing(self._ctx, 1 if enable else 0), "hj_ctx_set_timing")

    def last_timing(self):
        """ms of the last (init, build, probe, routing partition) launches and
        the probe's split into probe-side partitioning and the join kernel."""
        a = (C.c_float * 8)()
        check(lib.hj_ctx_last_timing_ex(self._ctx, a), "hj_ctx_last_timing_ex")
        return dict(zip(("init", "build", "probe", "partition", "probe_partition", "probe_join"), list(a)[:6]))

    def accumulate_timing(self, enable=True):
        """Per-step phase times with no host synchronisation between steps:
        each build starts a new event set (hj_ctx_timing_accumulate);
        timing_totals() sums them.  Enabling again drops what was recorded."""
        check(lib.hj_ctx_timing_accumulate(self._ctx, 1 if enable else 0), "hj_ctx_timing_accumulate")

    def timing_totals(self):
        """Summed ms of every build + probe step since accumulate_timing() or
        the last call (synchronises), with "steps": how many."""
        a = (C.c_float * 8)()
        n = C.c_longlong(0)
        check(lib.hj_ctx_timing_totals(self._ctx, a, C.byref(n)), "hj_ctx_timing_totals")
        d = dict(zip(("init", "build", "probe", "partition", "probe_partition", "probe_join"), list(a)[:6]))
        d["steps"] = n.value
        return d

    # -------------------------------------------------------------- phases
    def build_table(self, rkey, rpay=None, row_base=0, stream=None):
        """@initializeHashTable + @buildTable (join_v2.mlir:54-108)."""
        _need_cuda(rkey, rpay)
        st = _stream(self.device, stream)
        if rkey.dtype == torch.int64:
            if rpay is None or rpay.dtype != torch.int64 or rpay.numel() != rkey.numel():
                raise ValueError("int64 build needs an int64 payload column of the same length")
            check(lib.hj_dev_build_i64(self._ctx, _ptr(rkey), _ptr(rpay), rkey.numel(), st), "hj_dev_build_i64")
            self.key_bits = 64
        elif rkey.dtype == torch.int32:
            if rpay is not None:
                raise ValueError("i32 joins carry row ids, not payloads (reference types)")
            check(lib.hj_dev_build_i32(self._ctx, _ptr(rkey), rkey.numel(), int(row_base), st), "hj_dev_build_i32")
            self.key_bits = 32
        else:
            raise TypeError("keys must be int32 or int64")

    def build_tuples(self, tuples, stream=None):
        """Build from packed (n, 2) int64 {key, payload} rows (exchange format)."""
        _need_cuda(tuples)
        if tuples.dtype != torch.int64 or tuples.dim() != 2 or tuples.shape[1] != 2:
            raise ValueError("tuples must be an (n, 2) int64 tensor")
        check(lib.hj_dev_build_tuples_i64(self._ctx, _ptr(tuples), tuples.shape[0], _stream(self.device, stream)),
              "hj_dev_build_tuples_i64")
        self.key_bits = 64

    def count_rows(self, skey, stream=None, sync=True):
        """@countRows (join_v2.mlir:110-147): M, the result size."""
        _need_cuda(skey)
        st = _stream(self.device, stream)
        if skey.dtype == torch.int64:
            check(lib.hj_dev_count_i64(self._ctx, _ptr(skey), skey.numel(), _ptr(self._count), st), "hj_dev_count_i64")
        else:
            check(lib.hj_dev_count_i32(self._ctx, _ptr(skey), skey.numel(), _ptr(self._count), st), "hj_dev_count_i32")
        return int(self._count.item()) if sync else self._count

    def probe_relation(self, skey, spay=None, out_r=None, out_s=None, count=None, row_base=0, stream=None):
        """@probeRelation (join_v2.mlir:149-199).  Writes min(M, cap) rows into
        out_r / out_s; `count` (int64 device tensor) receives M.  Returns count."""
        _need_cuda(skey, spay, out_r, out_s)
        st = _stream(self.device, stream)
        count = self._count if count is None else count
        cap = 0 if out_r is None else out_r.numel()
        if out_s is not None and out_s.numel() != cap:
            raise ValueError("output columns differ in length")
        if skey.dtype == torch.int64:
            if spay is None or spay.dtype != torch.int64:
                raise ValueError("int64 probe needs an int64 payload column")
            check(lib.hj_dev_probe_i64(self._ctx, _ptr(skey), _ptr(spay), skey.numel(), _ptr(out_r), _ptr(out_s),
                                       cap, _ptr(count), st), "hj_dev_probe_i64")
        else:
            check(lib.hj_dev_probe_i32(self._ctx, _ptr(skey), skey.numel(), int(row_base), _ptr(out_r), _ptr(out_s),
                                       cap, _ptr(count), st), "hj_dev_probe_i32")
        return count

    def probe_tuples(self, tuples, out_r, out_s, count=None, stream=None):
        _need_cuda(tuples, out_r, out_s)
        count = self._count if count is None else count
        check(lib.hj_dev_probe_tuples_i64(self._ctx, _ptr(tuples), tuples.shape[0], _ptr(out_r), _ptr(out_s),
                                          out_r.numel(), _ptr(count), _stream(self.device, stream)),
              "hj_dev_probe_tuples_i64")
        return count

    # ---- folded routing (hj.h "Folded routing"): the owner and the
    # receiver's first radix-pass bin from one hash, so receivers skip a pass
    @staticmethod
    def route_plan(n_build_global, nranks):
        """Bin bits per owner for a routed join (0: no fold -- use partition)."""
        b = C.c_int(0)
        check(lib.hj_route_plan(int(n_build_global), int(nranks), C.byref(b)), "hj_route_plan")
        return b.value

    def route(self, key, pay, nranks, sub_bits, stream=None, slot=None):
        """(n, 2) tuples grouped by (owner, bin), and the (nranks << sub_bits)
        part sizes (int64 device tensor).  slot (e.g. "r" / "s"): the tuples
        go to a buffer this HashJoin keeps for that slot -- allocated once,
        placement-probed (placed_rows) -- and stay valid until the slot's next
        route; None: a fresh tensor."""
        _need_cuda(key, pay)
        n = key.shape[0]
        if slot is None:
            out = torch.empty((n, 2), dtype=torch.int64, device=self.device)
        else:
            buf = self._routed.get(slot)
            if buf is None or buf.shape[0] < n:
                self._routed.pop(slot, None)
                buf = placed_rows(n, self.device)
                self._routed[slot] = buf
            out = buf[:n]
        counts = torch.empty(nranks << sub_bits, dtype=torch.int64, device=self.device)
        check(lib.hj_dev_route_i64(self._ctx, _ptr(key), _ptr(pay), n, nranks, sub_bits, _ptr(out), _ptr(counts),
                                   _stream(self.device, stream)), "hj_dev_route_i64")
        return out, counts

    def build_routed(self, tuples, counts, nranks, sub_bits, stream=None):
        """Build from routed tuples; counts: (nsrc, 2^sub_bits) int64 device
        tensor of every source's bin sizes (rows laid out source by source)."""
        _need_cuda(tuples, counts)
        check(lib.hj_dev_build_routed_i64(self._ctx, _ptr(tuples), tuples.shape[0], _ptr(counts), counts.shape[0],
                                          nranks, sub_bits, _stream(self.device, stream)), "hj_dev_build_routed_i64")
        self.key_bits = 64

    def probe_routed(self, tuples, counts, bin0, out_r, out_s, count=None, stream=None):
        """Probe routed tuples of bins [bin0, bin0 + counts.shape[1])."""
        _need_cuda(tuples, counts, out_r, out_s)
        count = self._count if count is None else count
        check(lib.hj_dev_probe_routed_i64(self._ctx, _ptr(tuples), tuples.shape[0], _ptr(counts), counts.shape[0],
                                          bin0, counts.shape[1], _ptr(out_r), _ptr(out_s), out_r.numel(), _ptr(count),
                                          _stream(self.device, stream)), "hj_dev_probe_routed_i64")
        return count

    def partition(self, key, pay=None, nparts=2, out=None, counts=None, stream=None):
        """Radix-route rows to nparts owners: packed (n, 2) tuples grouped by
        owner + per-owner counts (int64 device tensor)."""
        st = _stream(self.device, stream)
        n = key.shape[0]
        out = torch.empty((n, 2), dtype=torch.int64, device=self.device) if out is None else out
        counts = torch.empty(nparts, dtype=torch.int64, device=self.device) if counts is None else counts
        if pay is None:   # key is already packed tuples
            _need_cuda(key, out, counts)
            check(lib.hj_dev_partition_tuples_i64(self._ctx, _ptr(key), n, nparts, _ptr(out), _ptr(counts), st),
                  "hj_dev_partition_tuples_i64")
        else:
            _need_cuda(key, pay, out, counts)
            check(lib.hj_dev_partition_i64(self._ctx, _ptr(key), _ptr(pay), n, nparts, _ptr(out), _ptr(counts), st),
                  "hj_dev_partition_i64")
        return out, counts

    # -------------------------------------------------------------- whole join
    def join_rows(self, t1, t2, stream=None):
        """nested-loop.mlir (:29-192) on device: t1, t2 are 2-D int32 tensors
        (row-major, key in column 0); returns the (M, c1 + c2 - 1) int32 rows
        [X row, Y cols 1..] of every key match, X the larger table (ties: t1).
        Count first, then materialise exactly M rows.  Row strides may exceed
        the column count (column slices of wider tables)."""
        for t in (t1, t2):
            if not t.is_cuda:
                raise ValueError("hash join inputs must be device tensors")
            if t.dtype != torch.int32 or t.dim() != 2 or (t.numel() and t.stride(1) != 1):
                raise ValueError("tables must be 2-D int32 tensors with unit column stride")
        ld = [t.stride(0) if t.numel() else t.shape[1] for t in (t1, t2)]
        st = _stream(self.device, stream)
        args = (_ptr(t1), t1.shape[0], t1.shape[1], ld[0], _ptr(t2), t2.shape[0], t2.shape[1], ld[1])
        check(lib.hj_dev_count_rows_i32(self._ctx, *args, _ptr(self._count), st), "hj_dev_count_rows_i32")
        m = int(self._count.item())
        oc = t1.shape[1] + t2.shape[1] - 1
        out = torch.empty((max(m, 1), oc), dtype=torch.int32, device=t1.device)
        check(lib.hj_dev_join_rows_i32(self._ctx, *args, _ptr(out), oc, m, _ptr(self._count), st),
              "hj_dev_join_rows_i32")
        return out[:m]

    def join_host(self, rkey, rpay, skey, spay, device_budget=0, capacity=None):
        """Out-of-core join of host-resident int64 numpy columns (relations
        larger than HBM): routed into groups that fit `device_budget` bytes
        (0 = 80 % of free HBM), each built on the GPU with its probe side
        streamed through.  Returns host arrays (R.pay, S.pay)."""
        import numpy as np
        cols = [np.ascontiguousarray(a, np.int64) for a in (rkey, rpay, skey, spay)]
        if cols[0].shape != cols[1].shape or cols[2].shape != cols[3].shape:
            raise ValueError("key and payload columns must have equal lengths")
        cap = max(1, cols[2].size if capacity is None else int(capacity))
        for _ in range(2):
            out_r = np.empty(cap, np.int64); out_s = np.empty(cap, np.int64)
            m = lib.hj_host_join_ooc_i64(self._ctx, cols[0].ctypes.data, cols[1].ctypes.data, cols[0].size,
                                         cols[2].ctypes.data, cols[3].ctypes.data, cols[2].size,
                                         out_r.ctypes.data, out_s.ctypes.data, cap, int(device_budget))
            if m < 0:
                check(int(m), "hj_host_join_ooc_i64")
            if m <= cap:
                return out_r[:m], out_s[:m]
            cap = int(m)
        raise RuntimeError("out-of-core join output did not fit after resizing")

    CMP = {"lt": 0, "le": 1, "gt": 2, "ge": 3, "eq": 4, "ne": 5}

    def select(self, values, op, value, with_rows=False, stream=None):
        """Experiments/selection.mlir's query on device: the elements v of a
        float32 or int64 tensor with `v <op> value` ('lt' 'le' 'gt' 'ge' 'eq'
        'ne'), compacted in input order (and their indices if with_rows)."""
        _need_cuda(values)
        if values.dtype not in (torch.float32, torch.int64) or values.dim() != 1:
            raise ValueError("selection input must be a 1-D float32 or int64 tensor")
        n = values.numel()
        out = torch.empty(max(n, 1), dtype=values.dtype, device=values.device)
        rows = torch.empty(max(n, 1), dtype=torch.int64, device=values.device) if with_rows else None
        f = lib.hj_dev_select_f32 if values.dtype == torch.float32 else lib.hj_dev_select_i64
        v = float(value) if values.dtype == torch.float32 else int(value)
        check(f(self._ctx, _ptr(values), n, self.CMP[op], v, _ptr(out), _ptr(rows) if with_rows else None, n,
                _ptr(self._count), _stream(self.device, stream)), "hj_dev_select")
        m = int(self._count.item())
        return (out[:m], rows[:m]) if with_rows else out[:m]

    def join(self, rkey, rpay, skey, spay=None, capacity=None, stream=None):
        """The @main join (join_v2.mlir:646-696) on device tensors: build, then
        probe into an output sized optimistically (|S| rows, or `capacity`),
        re-probing once at the exact M if that was too small."""
        self.probe_hint(skey.numel())
        try:
            self.build_table(rkey, rpay, stream=stream)
        finally:
            self.probe_hint(None)
        dt = torch.int64 if rkey.dtype == torch.int64 else torch.int32
        cap = max(1, skey.numel() if capacity is None else int(capacity))
        for _ in range(2):
            out_r = torch.empty(cap, dtype=dt, device=self.device)
            out_s = torch.empty(cap, dtype=dt, device=self.device)
            cnt = self.probe_relation(skey, spay, out_r, out_s, stream=stream)
            m = int(cnt.item())
            if m < 0:   # bit 63: an internal work list overflowed (hj.h)
                raise RuntimeError("hash join: internal work list overflow (count flagged)")
            if m <= cap:
                return out_r[:m], out_s[:m]
            cap = m
        raise RuntimeError("join output did not fit after resizing")


# ------------------------------------------------------------------ datagen
U64_MAX = (1 << 64) - 1


def hit_threshold(frac: float) -> int:
    if frac >= 1.0:
        return U64_MAX
    return min(U64_MAX - 1, int(frac * float(1 << 64)))


def gen_pkfk(seed, NR, NS, frac=1.0, r0=0, nr=None, s0=0, ns=None, device=None, stream=None):
    """Slice [r0, r0+nr) of R and [s0, s0+ns) of S of the PK-FK pair
    (SURVEY 8(d) C1/C3), generated on the device."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    nr = NR if nr is None else nr
    ns = NS if ns is None else ns
    rk = torch.empty(nr, dtype=torch.int64, device=dev); rp = torch.empty_like(rk)
    sk = torch.empty(ns, dtype=torch.int64, device=dev); sp = torch.empty_like(sk)
    check(lib.hj_dev_gen_pkfk_i64(seed, NR, hit_threshold(frac), r0, nr, _ptr(rk), _ptr(rp), s0, ns, _ptr(sk),
                                  _ptr(sp), _stream(dev, stream)), "hj_dev_gen_pkfk_i64")
    return rk, rp, sk, sp


def zipf_params(NR, theta):
    a = (C.c_double * 4)()
    check(lib.hj_zipf_params(int(NR), float(theta), a), "hj_zipf_params")
    return list(a)


def gen_zipf(seed, NR, NS, theta=0.9, s0=0, ns=None, device=None, stream=None):
    """Slice [s0, s0+ns) of a Zipf(theta) probe side over the PK-FK build side
    of the same seed (gen_pkfk's R), generated on the device."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    ns = NS if ns is None else ns
    sk = torch.empty(ns, dtype=torch.int64, device=dev); sp = torch.empty_like(sk)
    check(lib.hj_dev_gen_zipf_i64(seed, NR, float(theta), s0, ns, _ptr(sk), _ptr(sp), _stream(dev, stream)),
          "hj_dev_gen_zipf_i64")
    return sk, sp


def gen_uniform_i64(seed, stream_id, lo, hi, n, i0=0, device=None, stream=None):
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    k = torch.empty(n, dtype=torch.int64, device=dev); p = torch.empty_like(k)
    check(lib.hj_dev_gen_uniform_i64(seed, stream_id, lo, hi, i0, n, _ptr(k), _ptr(p), _stream(dev, stream)),
          "hj_dev_gen_uniform_i64")
    return k, p


def gen_uniform_i32(seed, stream_id, lo, hi, n, i0=0, device=None, stream=None):
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    k = torch.empty(n, dtype=torch.int32, device=dev)
    check(lib.hj_dev_gen_uniform_i32(seed, stream_id, lo, hi, i0, n, _ptr(k), _stream(dev, stream)),
          "hj_dev_gen_uniform_i32")
    return k


def device_info(device=0):
    """hipDeviceProp facts the roofline quotes (hj_device_info)."""
    a = (C.c_int64 * 8)()
    check(lib.hj_device_info(int(device), a), "hj_device_info")
    keys = ("cus", "memory_clock_khz", "memory_bus_bits", "l2_bytes", "hbm_bytes", "shader_clock_khz",
            "lds_bytes_per_cu", "peak_mb_per_s")
    return dict(zip(keys, [int(x) for x in a]))


COPY_SHAPES = {"persistent": 0, "flat": 1}


def stream_copy(src, dst, shape="persistent", stream=None):
    """Copy 16-B rows src -> dst on the device in one of the two reference
    copy shapes of hj_dev_stream_copy (the bench's copy floor)."""
    _need_cuda(src, dst)
    if src.numel() * src.element_size() != dst.numel() * dst.element_size() or src.numel() * src.element_size() % 16:
        raise ValueError("stream_copy needs equal-sized buffers of whole 16-B rows")
    rows = src.numel() * src.element_size() // 16
    check(lib.hj_dev_stream_copy(_ptr(src), _ptr(dst), rows, COPY_SHAPES[shape], _stream(src.device, stream)),
          "hj_dev_stream_copy")


# Routed-tuple buffers (the EXACT routing pass's destination) are drawn like
# the bucket sets' row buffers in libhj.so (hj_capi.cpp ensure_rows): a
# buffer of >= 1 GiB is probed (hj_placement_check: the partition pass's write
# pattern against a flat write) and redrawn while pattern/flat > 1.12 (the
# library's hj_placement_set_good value), up to 24 draws while free memory is
# >= 3x the buffer, holding at most 2 rejected draws at once (a further reject
# releases the oldest); the best draw is kept.  A buffer that keeps a slow
# draw is a give-up, counted in placement_stats().  HJ_PLACEMENT_PROBE=0
# turns it off.
PLACE_MIN_BYTES = 1 << 30
PLACE_DRAWS = 24
PLACE_HELD = 2
PLACE_SPARE = 3
_py_place = {"probes": 0, "rejected": 0, "gave_up": 0, "gave_up_low_mem": 0, "held_max": 0,
             "last_kept_ratio": 0.0, "worst_kept_ratio": 0.0}


def placed_rows(rows, device):
    """A (rows, 2) int64 device tensor at a placement the partition passes'
    write pattern runs fast in (see PLACE_*).

    The probe writes the candidate on the device's default HIP stream, so the
    caller's streams are drained first (a block torch hands out may still be
    in use by work queued on another stream).  Rejected draws are released to
    the driver with torch.cuda.empty_cache(), which also releases every other
    unused block torch has cached in this process (outside every timed
    region; the allocation is once per exchange buffer)."""
    rows = max(int(rows), 1)
    nbytes = rows * 16
    if nbytes < PLACE_MIN_BYTES or os.environ.get("HJ_PLACEMENT_PROBE", "1") == "0":
        return torch.empty((rows, 2), dtype=torch.int64, device=device)
    good = float(lib.hj_placement_set_good(0.0))
    torch.cuda.synchronize(device)
    held, best, best_r, draws, rejected, held_max, low_mem = [], None, float("inf"), 0, 0, 0, False
    for k in range(PLACE_DRAWS):
        if k > 0 and torch.cuda.mem_get_info(device)[0] < PLACE_SPARE * nbytes:
            low_mem = True
            break
        t = torch.empty((rows, 2), dtype=torch.int64, device=device)
        r = C.c_double(0.0)
        with torch.cuda.device(device):
            check(lib.hj_placement_check(_ptr(t), nbytes, C.byref(r)), "hj_placement_check")
        draws += 1
        if r.value < best_r:
            rej, best, best_r = best, t, r.value
        else:
            rej = t
        if rej is not None:
            rejected += 1
            held.append(rej)
            if len(held) > PLACE_HELD:
                held.pop(0)
            held_max = max(held_max, len(held))
        if best_r <= good:
            break
    _py_place["probes"] += draws
    _py_place["rejected"] += rejected
    if best_r > good:
        _py_place["gave_up"] += 1
        _py_place["gave_up_low_mem"] += int(low_mem)
    _py_place["held_max"] = max(_py_place["held_max"], held_max)
    _py_place["last_kept_ratio"] = round(best_r, 3)
    _py_place["worst_kept_ratio"] = max(_py_place["worst_kept_ratio"], round(best_r, 3))
    if rejected:
        del held, rej
        torch.cuda.empty_cache()   # the rejects go back to the driver, not to torch's cache
    return best


def placement_stats():
    """Row-buffer placement probe counts of this process (hj_placement_stats_ex):
    draws probed / rejected, buffers that kept a slow draw (gave_up; of those,
    gave_up_low_mem: free memory below 3x the buffer stopped the draws), the
    most rejected draws held at once, and the pattern/flat write ratio of the
    last and the worst buffer kept (~1.0 good, 1.25-1.35 a slow placement);
    routed_tuples: the same for the Python-drawn routed-tuple buffers."""
    out = (C.c_longlong * 5)()
    last, worst = C.c_double(0.0), C.c_double(0.0)
    lib.hj_placement_stats_ex(out, C.byref(last), C.byref(worst))
    return {"probes": out[0], "rejected": out[1], "gave_up": out[2], "gave_up_low_mem": out[3],
            "held_max": out[4], "last_kept_ratio": round(last.value, 3), "worst_kept_ratio": round(worst.value, 3),
            "routed_tuples": dict(_py_place)}


def partition_of(key: int, nparts: int) -> int:
    """Owner of a key under the routing hash (host function of libhj.so)."""
    return int(lib.hj_partition_of(int(key), int(nparts)))
