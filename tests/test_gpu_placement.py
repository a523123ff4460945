"""Placement probe of the large device buffers (hj_placement_check /
hj_placement_stats, hashjoin.placed_rows; DESIGN.md §2 "placement probe",
profiles/r05/placement.md).  The probe only chooses WHERE a buffer lives: the
join's results are the oracle-checked ones of the other GPU tests, here run
with the probe on (the default)."""
import ctypes as C

import pytest
import torch

import hashjoin
from hashjoin import join as J

pytestmark = pytest.mark.gpu


def test_placement_check_ratio():
    t = torch.empty((1 << 26, 2), dtype=torch.int64, device="cuda")   # 1 GiB
    r = C.c_double(0.0)
    assert hashjoin.lib.hj_placement_check(t.data_ptr(), t.numel() * 8, C.byref(r)) == 0
    # pattern / flat write time: ~1.0 good, 1.25-1.35 slow; never absurd
    assert 0.5 < r.value < 3.0


def test_placement_check_rejects_small_and_null():
    t = torch.empty(1 << 16, dtype=torch.int64, device="cuda")   # far below 256 buckets per CU
    r = C.c_double(0.0)
    assert hashjoin.lib.hj_placement_check(t.data_ptr(), t.numel() * 8, C.byref(r)) == -1
    assert hashjoin.lib.hj_placement_check(None, 1 << 30, C.byref(r)) == -1


def test_placed_rows_draws_and_counts():
    before = hashjoin.placement_stats()["routed_tuples"]["probes"]
    t = J.placed_rows(1 << 26, torch.device("cuda", 0))
    assert t.shape == (1 << 26, 2) and t.dtype == torch.int64 and t.is_cuda
    st = hashjoin.placement_stats()["routed_tuples"]
    assert st["probes"] > before
    assert 0.5 < st["last_kept_ratio"] < 3.0
    # small buffers are plain allocations, not probed
    s = J.placed_rows(1 << 10, torch.device("cuda", 0))
    assert s.shape == (1 << 10, 2)
    assert hashjoin.placement_stats()["routed_tuples"]["probes"] == st["probes"]


def test_bucket_sets_probed_and_join_exact():
    """A 2^26-row build allocates >= 512 MiB row buffers: they are probed, and
    the PK-FK join still returns every S row exactly once."""
    n = 1 << 26
    before = hashjoin.placement_stats()["probes"]
    rk, rp, sk, sp = hashjoin.gen_pkfk(7, n, n)
    hj = hashjoin.HashJoin(0)
    hj.set_strategy("radix")
    hj.allocate_hash_table(n, 64)
    hj.build_table(rk, rp)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == n
    st = hashjoin.placement_stats()
    assert st["probes"] > before
    assert st["rejected"] <= st["probes"]
    # every S row once (payload = row id for gen_pkfk's S side)
    assert torch.equal(torch.sort(out_s).values, torch.sort(sp).values)
    # each pair's R payload belongs to a row whose key equals the S row's key
    rkey_of = torch.empty_like(rk)
    rkey_of[rp] = rk
    skey_of = torch.empty_like(sk)
    skey_of[sp] = sk
    assert torch.equal(rkey_of[out_r], skey_of[out_s])
    hj.close()


def _c1_join(n=1 << 26, measure=False):
    """C1's PK-FK join on a fresh context; checks every S row once.  measure:
    also return the device memory the join holds at its end (inputs, outputs
    and the context's workspace)."""
    if measure:
        torch.cuda.empty_cache()   # (every tensor below then comes from the driver, and counts)
    free_a = torch.cuda.mem_get_info()[0]
    rk, rp, sk, sp = hashjoin.gen_pkfk(7, n, n)
    hj = hashjoin.HashJoin(0)
    try:
        hj.set_strategy("radix")
        hj.allocate_hash_table(n, 64)
        hj.build_table(rk, rp)
        out_r = torch.empty(n, dtype=torch.int64, device="cuda")
        out_s = torch.empty_like(out_r)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        assert int(cnt.item()) == n
        # every S row once (gen_pkfk's S payload is the row id: a permutation)
        seen = torch.zeros(n, dtype=torch.bool, device="cuda")
        seen[out_s] = True
        assert bool(seen.all())
        return free_a - torch.cuda.mem_get_info()[0] if measure else None
    finally:
        hj.close()


def test_placement_draws_bounded_and_give_up_reported():
    """with every draw judged slow (threshold forced
    down), each probed row buffer takes all 24 draws but never holds more than
    2 rejects at once, and keeps its best draw as a reported give-up; the
    Python-drawn routed-tuple buffers follow the same rules."""
    prev = hashjoin.lib.hj_placement_set_good(0.01)
    try:
        b = hashjoin.placement_stats()
        _c1_join()
        a = hashjoin.placement_stats()
        bufs = a["gave_up"] - b["gave_up"]
        assert bufs >= 1
        assert a["probes"] - b["probes"] == 24 * bufs
        assert a["held_max"] <= 2
        pb = a["routed_tuples"]
        t = J.placed_rows(1 << 26, torch.device("cuda", 0))
        assert t.shape == (1 << 26, 2)
        pa = hashjoin.placement_stats()["routed_tuples"]
        assert pa["probes"] - pb["probes"] == 24
        assert pa["gave_up"] == pb["gave_up"] + 1 and pa["held_max"] <= 2
    finally:
        hashjoin.lib.hj_placement_set_good(prev)
    assert abs(hashjoin.lib.hj_placement_set_good(0.0) - prev) < 1e-6


def test_placement_low_memory_join_gives_up_without_oom():
    """Most of HBM held by another allocation: the probe stops drawing once
    free memory falls below 3x a buffer (no OOM, no held rejects crowding the
    join out), the join is still exact, and the give-up is reported as a
    low-memory one."""
    free0 = torch.cuda.mem_get_info()[0]
    # the same join unconstrained: the memory it holds at its end (its
    # workspace goes back with its context, its tensors with empty_cache)
    used = _c1_join(measure=True)
    torch.cuda.empty_cache()
    # leave that plus 1 GiB: less than 3x any row buffer (2-3 GB each at
    # 2^26 rows) beyond what the join needs, so at least the last-allocated
    # buffers take one draw only
    need = used + (1 << 30)
    hold_bytes = torch.cuda.mem_get_info()[0] - need
    if hold_bytes <= 0:
        pytest.skip("device too small to leave a low-memory margin")
    hold = torch.empty(hold_bytes, dtype=torch.uint8, device="cuda")
    prev = hashjoin.lib.hj_placement_set_good(0.01)
    try:
        b = hashjoin.placement_stats()
        _c1_join()
        a = hashjoin.placement_stats()
        assert a["gave_up"] > b["gave_up"]
        assert a["gave_up_low_mem"] > b["gave_up_low_mem"]
        assert a["held_max"] <= 2
    finally:
        hashjoin.lib.hj_placement_set_good(prev)
        del hold
        torch.cuda.empty_cache()
    assert torch.cuda.mem_get_info()[0] > free0 // 2
