"""CPU tests of the C-ABI library: it loads, exports every symbol include/hj.h
declares, and its host-only logic behaves (no kernel launches here)."""
import ctypes as C
import subprocess

import numpy as np
import pytest

import hashjoin
from hashjoin import _lib


def test_exports_every_declared_symbol():
    names = hashjoin.declared_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(_lib.lib, n)]
    assert not missing, missing
    # and they are real dynamic exports of the .so
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [n for n in names if n not in exported]


def test_abi_version():
    assert hashjoin.lib.hj_abi_version() == 1


def test_built_for_gfx950_only():
    blob = open(_lib.LIB_PATH, "rb").read()
    import re
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def _np_partition_of(keys, P):
    k = keys.astype(np.uint64)
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xff51afd7ed558ccd)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xc4ceb9fe1a85ec53)
        k ^= k >> np.uint64(33)
        return (((k >> np.uint64(32)) * np.uint64(P)) >> np.uint64(32)).astype(np.int64)


@pytest.mark.parametrize("P", [1, 2, 3, 8, 1000])
def test_partition_of_matches_restatement(P):
    rng = np.random.default_rng(P)
    keys = np.concatenate([rng.integers(-(1 << 63), (1 << 63) - 1, 200, dtype=np.int64),
                           np.array([-(1 << 63), -1, 0, 1, (1 << 63) - 1], np.int64)])
    want = _np_partition_of(keys, P)
    got = np.array([hashjoin.partition_of(int(k), P) for k in keys])
    assert np.array_equal(got, want)
    assert got.min() >= 0 and got.max() < P


def test_partition_of_balanced():
    keys = np.arange(1 << 16, dtype=np.int64)
    counts = np.bincount(_np_partition_of(keys, 8), minlength=8)
    assert counts.max() / counts.mean() < 1.05


def test_memref_expansion_matches_lowered_abi():
    """5-scalar expansion (join_v1.ll:1262-1265) incl. offset/stride."""
    from hashjoin.memref import expand
    base = np.arange(20, dtype=np.int32)
    view = base[3:15:2]
    a = expand(view, base)
    assert a[0].value == base.ctypes.data and a[1].value == base.ctypes.data
    assert a[2:] == [3, 6, 2]


def test_errors_without_device_are_reported_not_fatal():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host-only check")
    ctx = hashjoin.lib.hj_ctx_create(0)
    assert not ctx
    assert b"device" in hashjoin.lib.hj_last_error()
    assert hashjoin.lib.hj_ctx_reserve(None, 10, 64) == _lib.HJ_ERR_ARG
    assert hashjoin.lib.hj_dev_probe_i64(None, None, None, 0, None, None, 0, None, None) == _lib.HJ_ERR_ARG


def test_header_compiles_as_c():
    src = '#include "hj.h"\nint main(void){ return hj_abi_version() == HJ_ABI_VERSION ? 0 : 1; }\n'
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", _lib.PKG_ROOT + "/../include",
                        "-x", "c", "-"], input=src, text=True, capture_output=True)
    assert r.returncode == 0, r.stderr


def test_reuse_mode_setter():
    """hj_host_set_reuse (host only): returns the previous mode, rejects
    unknown ones and leaves the mode unchanged then."""
    import hashjoin
    L = hashjoin.lib
    prev = L.hj_host_set_reuse(1)
    try:
        assert prev in (0, 1, 2)
        assert L.hj_host_set_reuse(2) == 1
        assert L.hj_host_set_reuse(7) == hashjoin._lib.HJ_ERR_ARG
        assert L.hj_host_set_reuse(0) == 2
    finally:
        L.hj_host_set_reuse(prev)


def test_route_plan_host():
    """The folded routing's bin bits (host function, no device needed): 9 -
    log2(ranks) bits below the owner bits while the local build side is
    radix-sized, 0 (route by owner only) otherwise."""
    import hashjoin
    rp = hashjoin.HashJoin.route_plan
    assert rp(1 << 28, 1) == 9 and rp(1 << 28, 2) == 8 and rp(1 << 28, 4) == 7 and rp(1 << 28, 8) == 6
    assert rp(1 << 28, 3) == 0            # not a power of two
    assert rp(1 << 20, 8) == 0            # 2^17 rows per rank: no radix build there
    assert rp(1 << 24, 1) == 9            # 2^24: 13 partition bits = 9 + 4
