"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

Small cases compare the exact sorted pair multiset with the oracle and the
golden fixtures (bit-exact; integer work has no tolerance).  Full-size cases
(BASELINE configs C1 / C1-ref / C2) use size-independent properties:
  * every output pair is a true match (R.key[r] == S.key[s], gathered on device),
  * no pair occurs twice,
  * the row count equals an independent count (sort + searchsorted),
which together force the output to be exactly the join's pair set.
"""
import numpy as np
import pytest
import torch

import hashjoin
from hashjoin import HashJoin
from hashjoin import memref as MR

from conftest import golden_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hj():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    h = HashJoin(0)
    yield h
    h.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def gpu_join(hj, rk, rp, sk, sp, capacity=None):
    if rk.dtype == np.int32:
        o_r, o_s = hj.join(dev(rk), None, dev(sk), None, capacity=capacity)
    else:
        o_r, o_s = hj.join(dev(rk), dev(rp), dev(sk), dev(sp), capacity=capacity)
    torch.cuda.synchronize()
    return host(o_r).astype(np.int64), host(o_s).astype(np.int64)


# ------------------------------------------------------------------ golden
@pytest.mark.parametrize("case", golden_cases())
def test_golden_device_api(hj, oracle, case):
    if int(case["kind"][0]) == 32:
        o = gpu_join(hj, case["r"], None, case["s"], None)
    else:
        o = gpu_join(hj, case["rk"], case["rp"], case["sk"], case["sp"])
    assert np.array_equal(oracle.sorted_pairs(*o), case["expected"])


@pytest.mark.parametrize("case", golden_cases())
def test_golden_memref_two_phase(oracle, case):
    """count -> alloc -> probe through the expanded memref ABI (join_v2.mlir:672-696)."""
    if int(case["kind"][0]) == 32:
        o_r, o_s = MR.join_i32_two_phase(case["r"], case["s"])
    else:
        rk, rp, sk, sp = case["rk"], case["rp"], case["sk"], case["sp"]
        m = MR.count_i64(rk, rp, sk, sp)
        assert m == len(case["expected"])
        o_r = np.empty(m, np.int64); o_s = np.empty(m, np.int64)
        assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
    assert np.array_equal(oracle.sorted_pairs(o_r, o_s), case["expected"])


@pytest.mark.parametrize("case", golden_cases())
def test_golden_ciface(oracle, case):
    """two-memref-in / one-memref-out C-interface entry points."""
    if int(case["kind"][0]) == 32:
        out = MR.ciface_join_i32(case["r"], case["s"])
    else:
        out = MR.ciface_join_kp_i64(case["rk"], case["rp"], case["sk"], case["sp"])
    assert out.shape == (len(case["expected"]), 2)
    assert np.array_equal(oracle.sorted_pairs(out[:, 0], out[:, 1]), case["expected"])


def test_ciface_i64_row_ids(oracle):
    rk, _ = oracle.gen_uniform_i64(5, 1, -30, 30, 700)
    sk, _ = oracle.gen_uniform_i64(5, 2, -30, 30, 900)
    out = MR.ciface_join_i64(rk, sk)
    exp = oracle.nested_loop_i64(rk, None, sk, None)
    assert oracle.same_multiset(out[:, 0], out[:, 1], *exp)


def test_memref_offsets_and_strides(oracle):
    base_r = oracle.gen_uniform_i32(1, 1, 1, 40, 3000)
    base_s = oracle.gen_uniform_i32(1, 2, 1, 40, 2000)
    r = base_r[5:2805:3]; s = base_s[1:1801:2]
    m = MR.count_i32(r, s, base_r, base_s)
    exp = oracle.nested_loop_i32(np.ascontiguousarray(r), np.ascontiguousarray(s))
    assert m == len(exp[0])
    # strided OUTPUT memrefs too
    o_r_base = np.full(2 * m + 1, -9, np.int32); o_s_base = np.full(2 * m + 1, -9, np.int32)
    assert MR.probe_i32(r, s, o_r_base[1::2], o_s_base[1::2]) == 0
    assert (o_r_base[0::2] == -9).all()
    assert oracle.same_multiset(o_r_base[1::2], o_s_base[1::2], *exp)
    # wrong output size is rejected
    assert MR.probe_i32(r, s, np.empty(m + 1, np.int32), np.empty(m + 1, np.int32)) == hashjoin._lib.HJ_ERR_CAPACITY


def test_memref_count_then_probe_reuses_the_join(oracle):
    """@countRows -> @probeRelation on the same inputs: the probe call returns
    the count call's pairs (no second build / probe); changed inputs at the
    same address get a fresh join (join_v1.mlir:110-176)."""
    r = oracle.gen_uniform_i32(9, 1, 1, 300, 20000)
    s = oracle.gen_uniform_i32(9, 2, 1, 300, 15000)
    h0 = hashjoin.lib.hj_host_memo_hits()
    m = MR.count_i32(r, s)
    o_r = np.empty(m, np.int32); o_s = np.empty(m, np.int32)
    assert MR.probe_i32(r, s, o_r, o_s) == 0
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 1
    assert oracle.same_multiset(o_r, o_s, *oracle.nested_loop_i32(r, s))
    s[:100] = 7                                  # same buffer, new contents
    m2 = MR.count_i32(r, s)
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 1
    exp2 = oracle.nested_loop_i32(r, s)
    assert m2 == len(exp2[0])
    o_r = np.empty(m2, np.int32); o_s = np.empty(m2, np.int32)
    assert MR.probe_i32(r, s, o_r, o_s) == 0
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 2
    assert oracle.same_multiset(o_r, o_s, *exp2)
    # i64 columns: reused too, and an i32 join in between invalidates nothing wrongly
    rk, rp, sk, sp = oracle.gen_pkfk_i64(12, 5000, 7000, 0.6)
    m3 = MR.count_i64(rk, rp, sk, sp)
    o_r = np.empty(m3, np.int64); o_s = np.empty(m3, np.int64)
    assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 3
    assert oracle.same_multiset(o_r, o_s, *oracle.nested_loop_i64(rk, rp, sk, sp))
    # inputs changed BETWEEN count and probe (same addresses, same sizes): the
    # probe's content digest differs, so it joins afresh instead of reusing
    m4 = MR.count_i64(rk, rp, sk, sp)
    sp[::7] += 1000                              # payloads only: same M, other pairs
    rk[3] = rk[4]                                # and a repeated build key
    exp4 = oracle.nested_loop_i64(rk, rp, sk, sp)
    o_r = np.empty(len(exp4[0]), np.int64); o_s = np.empty(len(exp4[0]), np.int64)
    assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 3
    assert oracle.same_multiset(o_r, o_s, *exp4)
    assert m4 >= 0
    # payloads changed, M the same: the probe's speculative delivery of the
    # kept pairs is overwritten by the fresh join's
    m5 = MR.count_i64(rk, rp, sk, sp)
    sp[::5] += 77
    exp5 = oracle.nested_loop_i64(rk, rp, sk, sp)
    assert len(exp5[0]) == m5
    o_r = np.empty(m5, np.int64); o_s = np.empty(m5, np.int64)
    assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
    assert hashjoin.lib.hj_host_memo_hits() == h0 + 3
    assert oracle.same_multiset(o_r, o_s, *exp5)


@pytest.mark.parametrize("mode", ["exact", "off"])
def test_memref_reuse_modes(oracle, mode):
    """hj_host_set_reuse: EXACT reuses only byte-identical inputs (a host copy
    kept by the count, compared with memcmp), OFF never reuses; both deliver
    the join of the probe's own inputs."""
    L = hashjoin.lib
    prev = L.hj_host_set_reuse({"exact": 1, "off": 2}[mode])
    try:
        rk, rp, sk, sp = oracle.gen_pkfk_i64(31, 6000, 9000, 0.7)
        h0 = L.hj_host_memo_hits()
        m = MR.count_i64(rk, rp, sk, sp)
        o_r = np.empty(m, np.int64); o_s = np.empty(m, np.int64)
        assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
        assert L.hj_host_memo_hits() == h0 + (1 if mode == "exact" else 0)
        assert oracle.same_multiset(o_r, o_s, *oracle.nested_loop_i64(rk, rp, sk, sp))
        # one payload byte changed between count and probe: never reused
        h1 = L.hj_host_memo_hits()
        m = MR.count_i64(rk, rp, sk, sp)
        sp[4321] ^= 1 << 40
        exp = oracle.nested_loop_i64(rk, rp, sk, sp)
        o_r = np.empty(len(exp[0]), np.int64); o_s = np.empty(len(exp[0]), np.int64)
        assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
        assert L.hj_host_memo_hits() == h1
        assert oracle.same_multiset(o_r, o_s, *exp)
        # strided i32 memrefs, unchanged: reused under EXACT
        base_r = oracle.gen_uniform_i32(32, 1, 1, 50, 4000)
        base_s = oracle.gen_uniform_i32(32, 2, 1, 50, 3000)
        r = base_r[3:3603:3]; s = base_s[1:2401:2]
        h2 = L.hj_host_memo_hits()
        m = MR.count_i32(r, s, base_r, base_s)
        o_r = np.empty(m, np.int32); o_s = np.empty(m, np.int32)
        assert MR.probe_i32(r, s, o_r, o_s) == 0
        assert L.hj_host_memo_hits() == h2 + (1 if mode == "exact" else 0)
        assert oracle.same_multiset(o_r, o_s, *oracle.nested_loop_i32(np.ascontiguousarray(r),
                                                                       np.ascontiguousarray(s)))
    finally:
        L.hj_host_set_reuse(prev)


def test_memref_concurrent_host_threads(oracle):
    """Host entry points share one default context: concurrent callers are
    serialised by its lock, each gets its own join."""
    import threading
    cases = [(oracle.gen_uniform_i32(20 + i, 1, 1, 200 + 50 * i, 6000 + 500 * i),
              oracle.gen_uniform_i32(20 + i, 2, 1, 200 + 50 * i, 5000 + 300 * i)) for i in range(6)]
    res = [None] * len(cases)

    def run(i):
        r, s = cases[i]
        for _ in range(3):
            out = MR.ciface_join_i32(r, s)
            res[i] = out

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for (r, s), out in zip(cases, res):
        assert oracle.same_multiset(out[:, 0], out[:, 1], *oracle.nested_loop_i32(r, s))


# ------------------------------------------------------------------ random vs oracle
CASES = [
    ("uniform_i64", 64, 5000, 7000, 1, 300),
    ("uniform_i64", 64, 1, 1, 1, 3),
    ("uniform_i64", 64, 1023, 1025, -5, 5),
    ("uniform_i64", 64, 20000, 30000, 1, 1 << 40),
    ("uniform_i32", 32, 4097, 3001, 1, 256),
    ("uniform_i32", 32, 20000, 20000, -(1 << 31), (1 << 31) - 1),
    ("uniform_i32", 32, 777, 5, 1, 2),
    ("pkfk", 64, 30000, 50000, 0, 0),
]


@pytest.mark.parametrize("kind,bits,nr,ns,lo,hi", CASES)
def test_random_vs_oracle(hj, oracle, kind, bits, nr, ns, lo, hi):
    if kind == "pkfk":
        rk, rp, sk, sp = oracle.gen_pkfk_i64(21, nr, ns, 0.6)
        rp = rp * 7 - 3
    elif bits == 64:
        rk, rp = oracle.gen_uniform_i64(nr + ns, 1, lo, hi, nr)
        sk, sp = oracle.gen_uniform_i64(nr + ns, 2, lo, hi, ns)
    else:
        rk = oracle.gen_uniform_i32(nr + ns, 1, lo, hi, nr); rp = None
        sk = oracle.gen_uniform_i32(nr + ns, 2, lo, hi, ns); sp = None
    o = gpu_join(hj, rk, rp, sk, sp)
    if bits == 64:
        exp = oracle.chained_join_i64(rk, rp, sk, sp, H=max(1, nr // 100))
    else:
        exp = oracle.chained_join_i32(rk, sk, H=max(1, nr // 100))
    assert oracle.same_multiset(*o, *exp)
    # count phase agrees
    if bits == 64:
        hj.build_table(dev(rk), dev(rp))
    else:
        hj.build_table(dev(rk))
    assert hj.count_rows(dev(sk)) == len(exp[0])


def test_empty_sides(hj, oracle):
    e64 = np.empty(0, np.int64)
    k, p = oracle.gen_uniform_i64(1, 1, 1, 10, 100)
    for rk, rp, sk, sp in [(e64, e64, k, p), (k, p, e64, e64), (e64, e64, e64, e64)]:
        hj.build_table(dev(rk) if len(rk) else torch.empty(0, dtype=torch.int64, device="cuda"),
                       dev(rp) if len(rp) else torch.empty(0, dtype=torch.int64, device="cuda"))
        out_r = torch.empty(4, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
        skd = dev(sk) if len(sk) else torch.empty(0, dtype=torch.int64, device="cuda")
        spd = dev(sp) if len(sp) else torch.empty(0, dtype=torch.int64, device="cuda")
        cnt = hj.probe_relation(skd, spd, out_r, out_s)
        assert int(cnt.item()) == 0


def test_int64_min_side_path(hj, oracle):
    """INT64_MIN is the table's EMPTY sentinel: such rows take the side list."""
    I64_MIN = -(1 << 63)
    rk = np.array([I64_MIN, 5, I64_MIN, 7, I64_MIN, 0], np.int64); rp = np.arange(6) * 10
    sk = np.array([I64_MIN, 7, 1, I64_MIN, 0], np.int64); sp = np.arange(5) + 100
    o = gpu_join(hj, rk, rp, sk, sp)
    assert oracle.same_multiset(*o, *oracle.nested_loop_i64(rk, rp, sk, sp))
    assert len(o[0]) == 3 * 2 + 1 + 1


def test_staging_overflow_many_matches_per_tile(hj, oracle):
    """> 1024 matches in one 1024-row tile: the spill-to-global path."""
    rk = np.repeat(np.arange(50, dtype=np.int64), 40)        # each key 40 times
    rp = np.arange(len(rk), dtype=np.int64)
    sk, sp = oracle.gen_uniform_i64(3, 2, 0, 49, 3000)      # every probe hits 40 rows
    o = gpu_join(hj, rk, rp, sk, sp)
    assert len(o[0]) == 3000 * 40
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=50))
    assert hj.has_duplicates()


def test_duplicate_flag(hj, oracle):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(4, 10000, 100, 1.0)
    hj.build_table(dev(rk), dev(rp))
    assert not hj.has_duplicates()
    rk2 = np.concatenate([rk, rk[:1]]); rp2 = np.concatenate([rp, [99999]])
    hj.build_table(dev(rk2), dev(rp2))
    assert hj.has_duplicates()


def test_capacity_too_small_reports_exact_count(hj, oracle):
    rk, _ = oracle.gen_uniform_i64(8, 1, 1, 20, 2000)
    sk, _ = oracle.gen_uniform_i64(8, 2, 1, 20, 2000)
    rp = np.arange(2000); sp = np.arange(2000)
    exp = oracle.nested_loop_i64(rk, rp, sk, sp)
    hj.build_table(dev(rk), dev(rp))
    cap = 1000
    out_r = torch.full((cap,), -1, dtype=torch.int64, device="cuda"); out_s = torch.full_like(out_r, -1)
    cnt = hj.probe_relation(dev(sk), dev(sp), out_r, out_s)
    assert int(cnt.item()) == len(exp[0])
    got = set(zip(host(out_r).tolist(), host(out_s).tolist()))
    assert (-1, -1) not in got and got <= set(zip(exp[0].tolist(), exp[1].tolist()))
    # the convenience join resizes and succeeds
    o = gpu_join(hj, rk, rp, sk, sp, capacity=10)
    assert oracle.same_multiset(*o, *exp)


def test_repeated_builds_reuse_context(hj, oracle):
    for seed in range(4):
        n = 1000 * (seed + 1)
        rk, rp, sk, sp = oracle.gen_pkfk_i64(seed, n, 2 * n, 0.5)
        o = gpu_join(hj, rk, rp, sk, sp)
        assert oracle.same_multiset(*o, *oracle.pkfk_expected(seed, n, 2 * n, 0.5))


# ------------------------------------------------------------------ datagen + partition
def test_datagen_matches_oracle(oracle):
    rk, rp, sk, sp = hashjoin.gen_pkfk(77, 5000, 6000, 0.7, r0=100, nr=3000, s0=50, ns=5000)
    want = oracle.gen_pkfk_i64(77, 5000, 6000, 0.7, 100, 3000, 50, 5000)
    for a, b in zip((rk, rp, sk, sp), want):
        assert np.array_equal(host(a), b)
    k, p = hashjoin.gen_uniform_i64(3, 9, -100, 1 << 50, 4000, i0=7)
    wk, wp = oracle.gen_uniform_i64(3, 9, -100, 1 << 50, 4000, i0=7)
    assert np.array_equal(host(k), wk) and np.array_equal(host(p), wp)
    k32 = hashjoin.gen_uniform_i32(3, 9, -(1 << 31), (1 << 31) - 1, 4000)
    assert np.array_equal(host(k32), oracle.gen_uniform_i32(3, 9, -(1 << 31), (1 << 31) - 1, 4000))


def test_partition_fanout_limit(hj):
    k = torch.arange(100, dtype=torch.int64, device="cuda")
    with pytest.raises(hashjoin.HJError):
        hj.partition(k, k, 8193)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8, 64, 65, 257, 1000, 4096, 8192])
def test_partition_kernel(hj, oracle, P):
    from test_abi import _np_partition_of
    k, p = oracle.gen_uniform_i64(P, 1, -(1 << 62), 1 << 62, 12345)
    k[:5] = -(1 << 63)
    out, counts = hj.partition(dev(k), dev(p), P)
    torch.cuda.synchronize()
    out = host(out); counts = host(counts)
    want_pid = _np_partition_of(k, P)
    assert np.array_equal(counts, np.bincount(want_pid, minlength=P))
    off = np.concatenate([[0], np.cumsum(counts)])
    for q in range(P):
        seg = out[off[q]:off[q + 1]]
        assert (_np_partition_of(seg[:, 0], P) == q).all()
    assert oracle.same_multiset(out[:, 0], out[:, 1], k, p)
    # packed-tuple input form routes identically
    out2, counts2 = hj.partition(torch.from_numpy(out).cuda(), None, P)
    assert np.array_equal(host(counts2), counts)


@pytest.mark.parametrize("P,n", [(8, 2048 * 5 + 77), (64, 2048 * 3), (4, 1), (6, 0)])
def test_partition_skewed_and_ragged(hj, oracle, P, n):
    """The 2048-row route tiles (4..64 parts): one hot key taking 3/4 of the
    rows, ragged and empty inputs; counts, owners and the multiset exact."""
    from test_abi import _np_partition_of
    k, p = oracle.gen_uniform_i64(P + 100, 2, -(1 << 62), 1 << 62, n)
    k[: (3 * n) // 4] = 12345
    out, counts = hj.partition(dev(k), dev(p), P)
    torch.cuda.synchronize()
    out = host(out); counts = host(counts)
    assert np.array_equal(counts, np.bincount(_np_partition_of(k, P), minlength=P))
    off = np.concatenate([[0], np.cumsum(counts)])
    for q in range(P):
        assert (_np_partition_of(out[off[q]:off[q + 1], 0], P) == q).all()
    assert oracle.same_multiset(out[:, 0], out[:, 1], k, p)


def test_tuple_build_probe(hj, oracle):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(31, 4000, 9000, 0.9)
    tr = dev(np.stack([rk, rp], 1)); ts = dev(np.stack([sk, sp], 1))
    hj.build_tuples(tr)
    out_r = torch.empty(9000, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    m = int(hj.probe_tuples(ts, out_r, out_s).item())
    assert oracle.same_multiset(host(out_r)[:m], host(out_s)[:m], *oracle.pkfk_expected(31, 4000, 9000, 0.9))


# ------------------------------------------------------------------ full size (BASELINE configs)
def _verify_pairs(rk, sk, o_r, o_s, r_is_row=True):
    """Every pair a true match, no pair twice; returns M."""
    m = o_r.numel()
    if m == 0:
        return 0
    assert bool((rk[o_r] == sk[o_s]).all())
    key = o_r * (sk.numel() + 1) + o_s
    assert torch.unique(key).numel() == m
    return m


def _independent_count(rk, sk):
    rs, _ = torch.sort(rk)
    lo = torch.searchsorted(rs, sk, side="left")
    hi = torch.searchsorted(rs, sk, side="right")
    return int((hi - lo).sum().item())


@pytest.mark.slow
def test_c1_pkfk_2p26(hj):
    n = 1 << 26
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
    hj.allocate_hash_table(n, 64)
    o_r, o_s = hj.join(rk, rp, sk, sp)
    assert o_r.numel() == n                                # f = 1: one match per probe row
    assert not hj.has_duplicates()
    assert _verify_pairs(rk, sk, o_r, o_s) == n
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))


@pytest.mark.slow
def test_c1ref_uniform_2p26(hj):
    n = 1 << 26
    rk, rp = hashjoin.gen_uniform_i64(0x5EED, 1, 1, 1 << 30, n)
    sk, sp = hashjoin.gen_uniform_i64(0x5EED, 2, 1, 1 << 30, n)
    o_r, o_s = hj.join(rk, rp, sk, sp)
    assert hj.has_duplicates()
    m = _verify_pairs(rk, sk, o_r, o_s)
    assert m == _independent_count(rk, sk)
    assert abs(m - (n * n) / (1 << 30)) < 0.01 * (n * n) / (1 << 30)


@pytest.mark.slow
def test_c2_small_build_huge_probe(hj):
    nr, ns = 1 << 20, 1 << 30
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, nr, ns)
    o_r, o_s = hj.join(rk, rp, sk, sp)
    assert o_r.numel() == ns
    # row-id payloads: every pair a true match, every S row exactly once
    assert bool((rk[o_r] == sk[o_s]).all())
    assert int(o_s.sum().item()) == ns * (ns - 1) // 2
    srt = torch.sort(o_s)[0]
    assert torch.equal(srt, torch.arange(ns, device="cuda"))


@pytest.mark.slow
def test_i32_reference_scale(hj):
    """join-performances.md:3 config shape at 1/10 size: 1M x 1M keys in [1, 100k] (M ~ 1e7)."""
    n = 1_000_000
    r = hashjoin.gen_uniform_i32(1, 1, 1, 100_000, n)
    s = hashjoin.gen_uniform_i32(1, 2, 1, 100_000, n)
    o_r, o_s = hj.join(r, None, s, None)
    m = o_r.numel()
    assert m == _independent_count(r.long(), s.long())
    assert bool((r[o_r.long()] == s[o_s.long()]).all())
    assert torch.unique(o_r.long() * n + o_s.long()).numel() == m


# ---------------------------------------------------------------- global table
# The global linear-probing table at oracle-checkable sizes: the fast path,
# the general path (duplicates, INT64_MIN keys) and the i32 layout.  (The
# XCD-split variant of this probe measured slower and was removed in round 4.)
@pytest.mark.parametrize("case", ["pkfk", "dups", "nulls", "i32"])
def test_global_table_vs_oracle(oracle, case):
    hj = HashJoin(0)
    try:
        hj.set_strategy("global")
        hj.set_timing(True)
        if case == "pkfk":
            rk, rp, sk, sp = oracle.gen_pkfk_i64(5, 100000, 300000, 0.7)
            exp = oracle.chained_join_i64(rk, rp, sk, sp, H=1000)
        elif case == "dups":
            rk, rp = oracle.gen_uniform_i64(6, 1, 1, 5000, 40000)
            sk, sp = oracle.gen_uniform_i64(6, 2, 1, 5000, 90000)
            exp = oracle.chained_join_i64(rk, rp, sk, sp, H=500)
        elif case == "nulls":
            rk, rp = oracle.gen_uniform_i64(7, 1, -200, 200, 20000)
            sk, sp = oracle.gen_uniform_i64(7, 2, -200, 200, 30000)
            rk[::101] = -(1 << 63); sk[::103] = -(1 << 63)
            exp = oracle.nested_loop_i64(rk, rp, sk, sp)
        else:
            r = oracle.gen_uniform_i32(8, 1, 1, 1 << 20, 50000)
            s = oracle.gen_uniform_i32(8, 2, 1, 1 << 20, 120000)
            o_r, o_s = hj.join(torch.from_numpy(r).cuda(), None, torch.from_numpy(s).cuda(), None)
            assert oracle.same_multiset(o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64),
                                        *oracle.chained_join_i32(r, s, H=1000))
            return
        d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (rk, rp, sk, sp)]
        o_r, o_s = hj.join(*d)
        assert hj.strategy_used == "global"
        assert oracle.same_multiset(o_r.cpu().numpy(), o_s.cpu().numpy(), *exp)
    finally:
        hj.close()


def test_memref_outputs_through_staging():
    """Outputs above the 16-MiB staging threshold (hj_capi.cpp d2h: 32-MiB
    page-locked chunks, several in flight, copied out by host threads) land
    intact in a contiguous and in a strided host memref: 2^22-row PK-FK
    (32 MiB per output column), every S row once with its R match."""
    n = 1 << 22
    rk, rp, sk, sp = (t.cpu().numpy() for t in hashjoin.gen_pkfk(99, n, n))
    m = MR.count_i64(rk, rp, sk, sp)
    assert m == n
    o_r = np.empty(m, np.int64)
    o_s = np.empty(m, np.int64)
    assert MR.probe_i64(rk, rp, sk, sp, o_r, o_s) == 0
    # gen_pkfk payloads are row ids: key of each pair's R and S row agree,
    # and every S row appears exactly once
    assert np.array_equal(np.sort(o_s), np.arange(n, dtype=np.int64))
    assert np.array_equal(rk[o_r], sk[o_s])
    # strided outputs (every other element of a 2m buffer) through the same path
    big_r = np.full(2 * m, -1, np.int64)
    big_s = np.full(2 * m, -1, np.int64)
    assert MR.probe_i64(rk, rp, sk, sp, big_r[::2], big_s[::2]) == 0
    assert np.array_equal(np.sort(big_s[::2]), np.arange(n, dtype=np.int64))
    assert np.array_equal(rk[big_r[::2]], sk[big_s[::2]])
    assert (big_r[1::2] == -1).all() and (big_s[1::2] == -1).all()
