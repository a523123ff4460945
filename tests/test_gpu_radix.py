"""GPU parity of the radix-partitioned strategy (hj_radix.hip) vs the oracle.

The partition count is forced (hj_ctx_set_radix_bits) so 1-, 2- and 3-pass
plans, empty partitions, oversized partitions (several LDS build rounds) and
the INT64_MIN side path are all exercised at sizes the oracle checks exactly.
"""
import numpy as np
import pytest
import torch

import hashjoin
from hashjoin import HashJoin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hj():
    h = HashJoin(0)
    yield h
    h.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run(hj, rk, rp, sk, sp, bits, capacity=None):
    hj.set_strategy("radix", radix_bits=bits)
    try:
        if rk.dtype == np.int32:
            o_r, o_s = hj.join(dev(rk), None, dev(sk), None, capacity=capacity)
        else:
            o_r, o_s = hj.join(dev(rk), dev(rp), dev(sk), dev(sp), capacity=capacity)
        assert hj.strategy_used == "radix"
        torch.cuda.synchronize()
        return o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64)
    finally:
        hj.set_strategy("auto")


@pytest.mark.parametrize("bits", [1, 3, 8, 9, 12, 16, 17])   # 1-pass ... 3-pass plans
def test_radix_pkfk_vs_oracle(hj, oracle, bits):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(bits, 20000, 30000, 0.7)
    o = run(hj, rk, rp * 5 - 1, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp * 5 - 1, sk, sp, H=200))


@pytest.mark.parametrize("bits", [2, 10])
def test_radix_duplicates_both_sides(hj, oracle, bits):
    rk, rp = oracle.gen_uniform_i64(bits, 1, 1, 500, 12000)
    sk, sp = oracle.gen_uniform_i64(bits, 2, 1, 500, 9000)
    o = run(hj, rk, rp, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=50))
    assert hj.has_duplicates()


def test_radix_oversized_partition_rounds(hj, oracle):
    """20000 build rows of ONE key land in one partition: > 5120 rows per LDS
    round, so the join runs several build rounds and still emits every pair."""
    rk = np.concatenate([np.full(20000, 42, np.int64), np.arange(1000, 3000, dtype=np.int64)])
    rp = np.arange(len(rk), dtype=np.int64)
    sk = np.array([42, 7, 42, 2500, 99999], np.int64); sp = np.arange(5, dtype=np.int64) + 10
    o = run(hj, rk, rp, sk, sp, 4)
    assert len(o[0]) == 2 * 20000 + 1
    assert oracle.same_multiset(*o, *oracle.nested_loop_i64(rk, rp, sk, sp))


def test_radix_big_probe_chunks(hj, oracle):
    """A hot probe key: one partition's S rows span many 8192-row chunks."""
    rk = np.arange(3000, dtype=np.int64) * 7; rp = np.arange(3000, dtype=np.int64)
    sk = np.concatenate([np.full(50000, 21, np.int64), np.arange(0, 30000, 3, dtype=np.int64)])
    sp = np.arange(len(sk), dtype=np.int64)
    o = run(hj, rk, rp, sk, sp, 6)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=300))


def test_radix_int64_min_keys(hj, oracle):
    I64_MIN = -(1 << 63)
    rk, rp = oracle.gen_uniform_i64(3, 1, -100, 100, 5000)
    sk, sp = oracle.gen_uniform_i64(3, 2, -100, 100, 4000)
    rk[::97] = I64_MIN; sk[::131] = I64_MIN
    o = run(hj, rk, rp, sk, sp, 5)
    assert oracle.same_multiset(*o, *oracle.nested_loop_i64(rk, rp, sk, sp))


@pytest.mark.parametrize("bits", [1, 9])
def test_radix_i32_reference_types(hj, oracle, bits):
    r = oracle.gen_uniform_i32(bits, 1, -(1 << 31), (1 << 31) - 1, 30000)
    s = np.concatenate([r[::3], oracle.gen_uniform_i32(bits, 2, 1, 1000, 10000)])
    o = run(hj, r, None, s, None, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i32(r, s, H=300))


def test_radix_empty_and_tiny(hj, oracle):
    e = np.empty(0, np.int64)
    k, p = oracle.gen_uniform_i64(1, 1, 1, 5, 10)
    for rk, rp, sk, sp in [(k, p, e, e), (e, e, k, p), (k[:1], p[:1], k[:1], p[:1])]:
        hj.set_strategy("radix", radix_bits=3)
        hj.build_table(torch.tensor(rk, dtype=torch.int64, device="cuda"), torch.tensor(rp, dtype=torch.int64, device="cuda"))
        out_r = torch.empty(64, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
        cnt = hj.probe_relation(torch.tensor(sk, dtype=torch.int64, device="cuda"),
                                torch.tensor(sp, dtype=torch.int64, device="cuda"), out_r, out_s)
        m = int(cnt.item())
        exp = oracle.nested_loop_i64(rk, rp, sk, sp)
        assert oracle.same_multiset(out_r.cpu().numpy()[:m], out_s.cpu().numpy()[:m], *exp)
    hj.set_strategy("auto")


def test_radix_count_and_capacity(hj, oracle):
    rk, rp = oracle.gen_uniform_i64(9, 1, 1, 2000, 40000)
    sk, sp = oracle.gen_uniform_i64(9, 2, 1, 2000, 40000)
    exp = oracle.nested_loop_i64(rk, rp, sk, sp)
    hj.set_strategy("radix", radix_bits=7)
    hj.build_table(dev(rk), dev(rp))
    assert hj.count_rows(dev(sk)) == len(exp[0])
    out_r = torch.empty(1000, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    assert int(hj.probe_relation(dev(sk), dev(sp), out_r, out_s).item()) == len(exp[0])
    hj.set_strategy("auto")
    o = run(hj, rk, rp, sk, sp, 7, capacity=5)
    assert oracle.same_multiset(*o, *exp)


@pytest.mark.parametrize("bits", [12, 17])
def test_radix_many_workgroups_vs_oracle(hj, oracle, bits):
    """2^20 rows: every workgroup owns many tiles and (pass 2) several
    segments, so open buckets are closed on segment switches and at the end;
    partitions are lists of full and partial buckets from several writers."""
    n = 1 << 20
    rk, rp, sk, sp = oracle.gen_pkfk_i64(bits + 100, n, n + 12345, 0.8)
    o = run(hj, rk, rp, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=n // 16))


def test_radix_unaligned_columns_and_tuples(hj, oracle):
    """Pass 1 reads two columns 16 B at a time when both are 16-B aligned;
    views offset by one element take the 8-B path.  Packed tuples too."""
    rk, rp, sk, sp = oracle.gen_pkfk_i64(77, 50001, 70003, 0.6)
    exp = oracle.chained_join_i64(rk[1:], rp[1:], sk[1:], sp[1:], H=500)
    R = [dev(rk), dev(rp)]; S = [dev(sk), dev(sp)]
    hj.set_strategy("radix", radix_bits=11)
    try:
        o_r, o_s = hj.join(R[0][1:], R[1][1:], S[0][1:], S[1][1:])
        assert R[0][1:].data_ptr() % 16 == 8
        assert oracle.same_multiset(o_r.cpu().numpy(), o_s.cpu().numpy(), *exp)
        tr = torch.stack([R[0][1:], R[1][1:]], 1).contiguous()
        ts = torch.stack([S[0][1:], S[1][1:]], 1).contiguous()
        hj.build_tuples(tr)
        assert hj.strategy_used == "radix"
        out_r = torch.empty(ts.shape[0], dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
        m = int(hj.probe_tuples(ts, out_r, out_s).item())
        assert oracle.same_multiset(out_r[:m].cpu().numpy(), out_s[:m].cpu().numpy(), *exp)
    finally:
        hj.set_strategy("auto")


def test_strategies_agree_full_size(hj):
    """C1 at 2^24: global and radix strategies give the same pair set."""
    n = 1 << 24
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n, 0.9)
    outs = []
    for strat in ("global", "radix"):
        hj.set_strategy(strat)
        o_r, o_s = hj.join(rk, rp, sk, sp)
        assert hj.strategy_used == strat
        order = torch.argsort(o_s)
        outs.append((o_r[order], o_s[order]))
    hj.set_strategy("auto")
    assert outs[0][0].numel() == outs[1][0].numel()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.slow
def test_radix_c3_2p28(hj):
    n = 1 << 28
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
    hj.set_strategy("radix")
    o_r, o_s = hj.join(rk, rp, sk, sp)
    hj.set_strategy("auto")
    assert o_r.numel() == n
    assert bool((rk[o_r] == sk[o_s]).all())
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))


def test_radix_many_subchunk_items(hj, oracle):
    """Small R, long S: each work item probes one LDS table with many
    2560-row sub-chunks, and a partition's S spans several items."""
    rk, rp, sk, sp = oracle.gen_pkfk_i64(31, 3000, 400000, 0.9)
    o = run(hj, rk, rp, sk, sp, 1)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=300))


def test_auto_probe_time_strategy(hj):
    """AUTO with a build side in [2^18, 2^21): the global table is built AND
    R is radix-partitioned; a probe side >= 2^24 rows takes the radix join,
    a smaller one the global table -- same pairs either way."""
    nr = 1 << 18
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, nr, 1 << 24, 0.95)
    hj.set_strategy("auto")
    res = {}
    for ns in (1 << 20, 1 << 24):
        o_r, o_s = hj.join(rk, rp, sk[:ns], sp[:ns])
        res[ns] = hj.strategy_used
        order = torch.argsort(o_s)
        hj.set_strategy("global")
        g_r, g_s = hj.join(rk, rp, sk[:ns], sp[:ns])
        hj.set_strategy("auto")
        gorder = torch.argsort(g_s)
        assert o_r.numel() == g_r.numel()
        assert torch.equal(o_r[order], g_r[gorder]) and torch.equal(o_s[order], g_s[gorder])
    assert res == {1 << 20: "global", 1 << 24: "radix"}


def test_auto_probe_hint(hj):
    """hj_ctx_probe_hint: a probe side known to stay below 2^24 rows spares a
    [2^18, 2^21)-row AUTO build its radix partition (no plan); a later, larger
    probe still joins -- through the global table, with the pairs of a
    forced-global join."""
    nr, ns = 1 << 18, 1 << 24
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EEE, nr, ns, 0.95)
    hj.set_strategy("auto")
    try:
        hj.probe_hint(None)
        hj.build_table(rk, rp)
        assert hj.radix_plan   # unknown probe side: R partitioned as well
        hj.probe_hint(1 << 20)
        hj.build_table(rk, rp)
        assert not hj.radix_plan
        out_r = torch.empty(ns, dtype=torch.int64, device="cuda")
        out_s = torch.empty_like(out_r)
        m = int(hj.probe_relation(sk, sp, out_r, out_s).item())
        assert hj.strategy_used == "global"
        hj.probe_hint(None)
        hj.set_strategy("global")
        g_r, g_s = hj.join(rk, rp, sk, sp)
        assert m == g_r.numel()
        o_r, o_s = out_r[:m], out_s[:m]
        order, gorder = torch.argsort(o_s), torch.argsort(g_s)
        assert torch.equal(o_r[order], g_r[gorder]) and torch.equal(o_s[order], g_s[gorder])
    finally:
        hj.probe_hint(None)
        hj.set_strategy("auto")


@pytest.mark.parametrize("bits", [9, 17])
def test_radix_hot_key_tiles_i32(hj, oracle, bits):
    """The same skew on the reference types (i32 keys, row-id payloads)."""
    rng = np.random.default_rng(18)
    r = (np.arange(65536, dtype=np.int64) * 7 - 200000).astype(np.int32)
    n = 1 << 20
    u = rng.random(n)
    s = np.where(u < 0.45, r[3], np.where(u < 0.55, r[40000], r[rng.integers(0, 65536, n)])).astype(np.int32)
    o = run(hj, r, None, s, None, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i32(r, s, H=4096))


@pytest.mark.parametrize("bits", [9, 17])
def test_radix_hot_key_tiles(hj, oracle, bits):
    """Skewed probe keys: 40 % / 10 % of 2^20 S rows carry two hot keys, so
    most tiles of a workgroup (>= 8 each) hold a bin of > kTile / 8 rows and
    k_pass counts that bin's lanes with one atomic per wave instruction."""
    rng = np.random.default_rng(17)
    rk = np.arange(65536, dtype=np.int64) * 7; rp = np.arange(65536, dtype=np.int64) + 3
    n = 1 << 20
    u = rng.random(n)
    sk = np.where(u < 0.4, 21, np.where(u < 0.5, 70, rng.integers(0, 65536 * 7, n))).astype(np.int64)
    sp = np.arange(n, dtype=np.int64)
    o = run(hj, rk, rp, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=4096))


@pytest.mark.parametrize("bits", [12, 17])
def test_radix_heavy_items_first(hj, oracle, bits):
    """Half of 2^21 S rows on 40 hot keys of Zipf-like weights: their
    partitions split into several work items each (the rest one item), and
    the join lists those items first (k_item_desc's heavy-first order) --
    every pair still comes out exactly once."""
    rng = np.random.default_rng(23)
    rk = np.arange(1 << 16, dtype=np.int64) * 11 + 5
    rp = np.arange(1 << 16, dtype=np.int64) - 9
    n = 1 << 21
    w = 1.0 / np.arange(1, 41) ** 0.9
    hot = rng.choice(rk, 40, replace=False)
    u = rng.random(n)
    sk = np.where(u < 0.5, hot[rng.choice(40, n, p=w / w.sum())], rk[rng.integers(0, 1 << 16, n)]).astype(np.int64)
    sp = np.arange(n, dtype=np.int64) * 3
    o = run(hj, rk, rp, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=4096))


@pytest.mark.parametrize("bits", [3, 7])
def test_radix_i32_many_matches_per_row(hj, oracle, bits):
    """~100 build copies per key (the reference's 10M x 10M / [1, 100k] shape,
    scaled down): sub-chunks with > 2 matches per probe row take the wave-
    cooperative write path; pairs must equal the oracle's."""
    r = oracle.gen_uniform_i32(70 + bits, 1, 1, 400, 40000)
    s = oracle.gen_uniform_i32(70 + bits, 2, 1, 400, 30000)
    s[:7] = 999                     # no match
    o = run(hj, r, None, s, None, bits)
    exp = oracle.chained_join_i32(r, s, H=400)
    assert len(o[0]) == len(exp[0]) > 2 * len(s)
    assert oracle.same_multiset(*o, exp[0].astype(np.int64), exp[1].astype(np.int64))


def test_radix_i32_grouped_join_counts_capacity_and_repeats(oracle):
    """Repeated i32 keys (~80 copies each, keys incl. -1 and INT32_MIN) on
    one context, joined many times: the first join's fast path defers the
    items to the grouped join (k_join_grp, list mode), the following ones run
    it over every item; count-only calls, an output far smaller than M (the
    count is still M, the rows written are true, distinct pairs) and a
    resize-and-retry join must all agree with the oracle."""
    r = oracle.gen_uniform_i32(81, 1, 1, 300, 24000)
    s = oracle.gen_uniform_i32(81, 2, 1, 300, 18000)
    r[:80] = -1; s[:5] = -1
    r[80:160] = -(1 << 31); s[5:9] = -(1 << 31)
    s[9:20] = 12345                   # no match
    exp = oracle.chained_join_i32(r, s, H=300)
    m = len(exp[0])
    assert m > 50 * len(s)
    h = HashJoin(0)
    try:
        h.set_strategy("radix", radix_bits=6)
        for i in range(4):
            h.build_table(dev(r), None)
            assert h.count_rows(dev(s)) == m, f"count {i}"
            out_r = torch.empty(1000, dtype=torch.int32, device="cuda"); out_s = torch.empty_like(out_r)
            assert int(h.probe_relation(dev(s), None, out_r, out_s).item()) == m, f"probe {i}"
            pr, ps = out_r.cpu().numpy().astype(np.int64), out_s.cpu().numpy().astype(np.int64)
            assert (r[pr] == s[ps]).all() and len(set(zip(pr.tolist(), ps.tolist()))) == 1000, f"truncated {i}"
            o_r, o_s = h.join(dev(r), None, dev(s), None, capacity=7)
            torch.cuda.synchronize()
            assert oracle.same_multiset(o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64),
                                        exp[0].astype(np.int64), exp[1].astype(np.int64)), f"join {i}"
        assert h.has_duplicates()
        # the context now runs the grouped join on every narrow item: distinct
        # keys at ~4000 build rows per partition (near-full 4096-slot tables,
        # the largest items deferred on to k_join) and probes that miss
        ru = np.random.default_rng(5).permutation(1 << 20)[:64000].astype(np.int32) * 3 + 1
        su = np.concatenate([ru[::2], ru[1::7] + 1]).astype(np.int32)
        h.set_strategy("radix", radix_bits=4)
        o_r, o_s = h.join(dev(ru), None, dev(su), None)
        torch.cuda.synchronize()
        ex = oracle.chained_join_i32(ru, su, H=1000)
        assert oracle.same_multiset(o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64),
                                    ex[0].astype(np.int64), ex[1].astype(np.int64))
    finally:
        h.close()


def test_join_kernel_choice_is_deterministic(oracle):
    """The join kernel is a function of the data (row width, probe / build
    ratio, the build side's sampled repeats), never of an earlier join on the
    context: interleaved joins of different shapes each get their own kernel,
    the same join run twice back to back gets the same one, and every result
    equals the oracle."""
    h = HashJoin(0)
    try:
        h.set_strategy("radix", radix_bits=6)
        # i32, ~40 copies of every key (REF-A's shape): the grouped join
        rk = oracle.gen_uniform_i64(7, 1, 1, 400, 16000)[0].astype(np.int32)
        sk = oracle.gen_uniform_i64(7, 2, 1, 400, 12000)[0].astype(np.int32)
        exp = oracle.chained_join_i32(rk, sk, H=64)
        # i64 PK-FK: the bucketed table
        pk_r, pk_p, pk_s, pk_sp = oracle.gen_pkfk_i64(6, 20000, 30000, 0.9)
        exp_pk = oracle.chained_join_i64(pk_r, pk_p, pk_s, pk_sp, H=200)
        # i64, a repeated key in every tenth build row: still the bucketed
        # table (its marked-slot multi-match path)
        dk, dp = oracle.gen_uniform_i64(8, 1, 1, 1 << 40, 20000)
        dk = dk.copy()
        dk[::10] = dk[1::10]
        sk64, sp64 = oracle.gen_uniform_i64(8, 2, 1, 1 << 40, 20000)
        sk64 = sk64.copy()
        sk64[:5000] = dk[:5000]
        exp_d = oracle.chained_join_i64(dk, dp, sk64, sp64, H=200)
        # i64, keys in [1, 2000] (~90 % of the build rows repeat): the grouped join over every item
        hk, hp = oracle.gen_uniform_i64(10, 1, 1, 2000, 20000)
        hs, hsp = oracle.gen_uniform_i64(10, 2, 1, 2000, 6000)
        exp_h = oracle.chained_join_i64(hk, hp, hs, hsp, H=200)
        # i32 unique-ish keys: k_join_b (keys and row ids apart)
        uk = oracle.gen_uniform_i64(9, 1, 1, 1 << 30, 20000)[0].astype(np.int32)
        us = oracle.gen_uniform_i64(9, 2, 1, 1 << 30, 20000)[0].astype(np.int32)
        us[:4000] = uk[:4000]
        exp_u = oracle.chained_join_i32(uk, us, H=200)

        def i32(a, b, want):
            o_r, o_s = h.join(dev(a), None, dev(b), None)
            torch.cuda.synchronize()
            assert oracle.same_multiset(o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64),
                                        want[0].astype(np.int64), want[1].astype(np.int64))
            return h.join_kernel

        def i64(rk_, rp_, sk_, sp_, want):
            o_r, o_s = h.join(dev(rk_), dev(rp_), dev(sk_), dev(sp_))
            torch.cuda.synchronize()
            assert oracle.same_multiset(o_r.cpu().numpy(), o_s.cpu().numpy(), *want)
            return h.join_kernel

        seq = [("grp", lambda: i32(rk, sk, exp)), ("grp", lambda: i32(rk, sk, exp)),
               ("b", lambda: i64(pk_r, pk_p, pk_s, pk_sp, exp_pk)), ("u", lambda: i64(dk, dp, sk64, sp64, exp_d)),
               ("b", lambda: i64(pk_r, pk_p, pk_s, pk_sp, exp_pk)), ("u32", lambda: i32(uk, us, exp_u)),
               ("grp", lambda: i32(rk, sk, exp)), ("u", lambda: i64(dk, dp, sk64, sp64, exp_d)),
               ("u", lambda: i64(dk, dp, sk64, sp64, exp_d)), ("b", lambda: i64(pk_r, pk_p, pk_s, pk_sp, exp_pk)),
               ("g", lambda: i64(hk, hp, hs, hsp, exp_h)), ("u32", lambda: i32(uk, us, exp_u)),
               ("g", lambda: i64(hk, hp, hs, hsp, exp_h))]
        want_k = {"grp": "k_join_grp", "b": "k_join_b", "u": "k_join_b", "u32": "k_join_b", "g": "k_join_grp"}
        for i, (what, fn) in enumerate(seq):
            assert fn() == want_k[what], f"join {i} ({what})"
    finally:
        h.close()


@pytest.mark.parametrize("dist", ["pkfk", "dups"])
def test_radix_probe_heavy_stream_shape(hj, oracle, dist):
    """A probe side >= 8x the build side takes the fast join's stream shape
    (1024 threads, 4 probe rows per thread, many sub-chunks per item)."""
    if dist == "pkfk":
        rk, rp, sk, sp = oracle.gen_pkfk_i64(11, 6000, 90000, 0.8)
    else:
        rk, rp = oracle.gen_uniform_i64(11, 1, 1, 3000, 6000)
        sk, sp = oracle.gen_uniform_i64(11, 2, 1, 3000, 90000)
    o = run(hj, rk, rp, sk, sp, 3)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=300))
    assert hj.join_kernel == "k_join_u_stream"


@pytest.mark.parametrize("rows,bits", [(200000, 7), (180000, 6)])
@pytest.mark.parametrize("dups", ["none", "one", "hot", "unprobed"])
def test_radix_bucketed_table_repeat_detection(hj, oracle, rows, bits, dups):
    """The wide fast join's bucketed table (k_join_b): a probe row that meets
    a repeated build key flags the repeat during the join, and the rest of the
    exact answer comes from the on-demand check (k_join_b DETECT: signature
    suspects + a chain check) -- no repeat among unique keys at ~1500 and
    ~2800 rows per partition (the second crowds buckets into overflow
    chains), one repeated pair, one key 40 times (its copies fill its home
    bucket and spill over), and repeats no probe row meets."""
    rk, rp, sk, sp = oracle.gen_pkfk_i64(rows + bits, rows, rows, 0.8)
    rk = rk.copy()
    if dups == "one":
        rk[7] = rk[12345]
    elif dups == "hot":
        rk[100:140] = rk[99]
    elif dups == "unprobed":
        rk[7] = rk[12345]
        rk[100:140] = rk[99]
        sk = sk.copy()
        sk[np.isin(sk, rk[[7, 99]])] = -5   # (the oracle joins it like any key)
    o = run(hj, rk, rp, sk, sp, bits)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=1000))
    assert hj.has_duplicates() == (dups != "none")


def test_wide_join_choice_after_repeats(oracle):
    """int64 joins alternating between build sides with repeated keys in
    every partition (k_join_b's multi-match path) and unique keys: results
    and the repeat flag stay exact across the switches."""
    h = HashJoin(0)
    try:
        rk_u, rp_u, sk_u, sp_u = oracle.gen_pkfk_i64(41, 150000, 150000, 0.9)
        rk_d, rp_d = oracle.gen_uniform_i64(42, 1, 1, 1 << 30, 150000)
        sk_d, sp_d = oracle.gen_uniform_i64(42, 2, 1, 1 << 30, 150000)
        rk_d[:3000] = rk_d[3000:6000]   # some repeats in every partition
        want_u = oracle.chained_join_i64(rk_u, rp_u, sk_u, sp_u, H=1000)
        want_d = oracle.chained_join_i64(rk_d, rp_d, sk_d, sp_d, H=1000)
        for i, dup in enumerate([True, False, False, True] + [False] * 6):
            rk, rp, sk, sp, want = (rk_d, rp_d, sk_d, sp_d, want_d) if dup else (rk_u, rp_u, sk_u, sp_u, want_u)
            o = run(h, rk, rp, sk, sp, 6)
            assert oracle.same_multiset(*o, *want), f"join {i}"
            assert h.has_duplicates() == dup, f"join {i}"
            assert h.join_kernel == "k_join_b", f"join {i}"
    finally:
        h.close()


@pytest.mark.parametrize("wide", [True, False])
@pytest.mark.parametrize("pattern", ["pairs", "mixed", "hot", "overflow"])
def test_radix_bucketed_multi_match(hj, oracle, wide, pattern):
    """k_join_b's repeated build keys: every copy of a repeated key is marked
    by the suspects' chain checks, and probe rows whose first match is marked
    write all their pairs by a chain walk -- pairs (2 copies), a mix of 2..6
    copies (C1-ref-like), one key 40x, and copies crowding home buckets past
    their 4 slots (chains over several buckets).  int64 rows; the same
    shapes with i32 rows (keys and row ids in separate LDS arrays)."""
    n = 60000
    rng = np.random.default_rng(1234 + len(pattern) + (7 if wide else 0))
    base = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=n, replace=False)
    rk = base.copy()
    # (repeats stay under a quarter of the build rows: the sample then keeps
    # k_join_b, asserted below)
    if pattern == "pairs":
        rk[1:n // 4:2] = rk[0:n // 4:2][: len(rk[1:n // 4:2])]
    elif pattern == "mixed":
        reps = rng.integers(1, 7, size=n // 8)
        rk[: n // 8] = np.repeat(base[n // 8: n // 4], reps)[: n // 8]
    elif pattern == "hot":
        rk[500:540] = rk[499]
    else:   # keys crowding one home bucket region: many copies of few keys
        rk[:4000] = np.repeat(base[:400], 10)
    rng.shuffle(rk)
    sk = np.concatenate([rng.choice(rk, size=n // 2), rng.integers(1, 1 << 30, size=n // 2)])
    rp = np.arange(n, dtype=np.int64) * 3 + 1
    sp = np.arange(len(sk), dtype=np.int64) * 5 + 2
    if wide:
        o = run(hj, rk, rp, sk, sp, 6)
        assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=1000))
    else:
        o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 6)
        ex = oracle.chained_join_i32(rk.astype(np.int32), sk.astype(np.int32), H=1000)
        assert oracle.same_multiset(*o, ex[0].astype(np.int64), ex[1].astype(np.int64))
    assert hj.has_duplicates()
    assert hj.join_kernel == "k_join_b"


@pytest.mark.parametrize("dups", [False, True])
def test_radix_narrow_unprobed_repeats(hj, oracle, dups):
    """i32 rows through k_join_b: a repeated build key that no probe row meets
    is still reported (the on-demand DETECT build), and unique keys are not."""
    n = 120000
    rng = np.random.default_rng(77)
    rk = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=n, replace=False)
    if dups:
        rk[5] = rk[77]
        rk[1000:1030] = rk[999]
    sk = np.concatenate([rng.choice(rk, size=n // 2), rng.integers(1, 1 << 30, size=n // 2)])
    sk[np.isin(sk, rk[[5, 999]])] = 3   # (the oracle joins it like any key)
    o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 6)
    ex = oracle.chained_join_i32(rk.astype(np.int32), sk.astype(np.int32), H=1000)
    assert oracle.same_multiset(*o, ex[0].astype(np.int64), ex[1].astype(np.int64))
    assert hj.join_kernel == "k_join_b"
    assert hj.has_duplicates() == dups


@pytest.mark.parametrize("wide", [True, False])
def test_radix_detect_many_suspects(hj, oracle, wide):
    """The on-demand repeat check when one partition holds more suspects than
    k_join_b's suspect list (512): every live slot of that table checks its
    chain instead.  Partition 0 of a 6-bit plan gets 40 keys x 25 copies on
    top of its share of unique keys (~2560 rows, under the 3/4-table defer
    limit); no probe row meets a repeated key, so only the check can report
    them."""
    rng = np.random.default_rng(4242)
    cand = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=400000, replace=False)
    top6 = ((cand.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(58)).astype(np.int64)
    hot = cand[top6 == 0][:40]
    rest = cand[top6 != 0]
    uniq = np.concatenate([cand[top6 == 0][40:40 + 1560], rest[:98440]])
    rk = np.concatenate([uniq, np.repeat(hot, 25)])
    rng.shuffle(rk)
    sk = np.concatenate([rng.choice(uniq, size=60000), rng.integers(1 << 30, 1 << 31, size=20000)])
    rp = np.arange(len(rk), dtype=np.int64) * 7 + 3
    sp = np.arange(len(sk), dtype=np.int64) * 11 + 5
    if wide:
        o = run(hj, rk, rp, sk, sp, 6)
        assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=1000))
    else:
        o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 6)
        ex = oracle.chained_join_i32(rk.astype(np.int32), sk.astype(np.int32), H=1000)
        assert oracle.same_multiset(*o, ex[0].astype(np.int64), ex[1].astype(np.int64))
    assert hj.join_kernel == "k_join_b"
    assert hj.has_duplicates()


def _fuzz_cases():
    """Seeded sizes just around the kernels' units (64-row runs, 512/1024-row
    buckets, 4096-row pass tiles, 8192-row probe chunks), key ranges from
    every-key-repeats to nearly unique, both row widths, 1-3 pass plans."""
    rng = np.random.default_rng(0x5eed)
    units = [1, 63, 64, 65, 511, 513, 1023, 1025, 4095, 4096, 4097, 8191, 8193, 12289, 40961]
    cases = []
    for i in range(24):
        nr = int(rng.choice(units)) + int(rng.integers(0, 3))
        ns = int(rng.choice(units)) * int(rng.integers(1, 4))
        span = int(rng.choice([3, 64, 1000, 1 << 20, 1 << 40]))
        span = max(span, nr * ns // 2_000_000 + 1)   # at most ~2M result rows
        bits = int(rng.choice([1, 4, 7, 9, 12, 17]))
        wide = bool(i % 3)
        cases.append((i, nr, ns, span if wide else min(span, 1 << 30), bits, wide))
    return cases


def _fuzz_keys(rng, lo, span, nr, ns):
    # ~70 % of S rows take a key drawn from R (sparse spans still match)
    rk = rng.integers(lo, lo + span, nr, dtype=np.int64)
    sk = rng.integers(lo, lo + span, ns, dtype=np.int64)
    hit = rng.random(ns) < 0.7
    sk[hit] = rk[rng.integers(0, nr, int(hit.sum()))]
    return rk, sk


@pytest.mark.parametrize("i,nr,ns,span,bits,wide", _fuzz_cases())
def test_radix_fuzz_ragged_vs_oracle(hj, oracle, i, nr, ns, span, bits, wide):
    rng = np.random.default_rng(1000 + i)
    lo = -span // 2
    if wide:
        rk, sk = _fuzz_keys(rng, lo, span, nr, ns)
        rp = rng.integers(-(1 << 62), 1 << 62, nr, dtype=np.int64)
        sp = rng.integers(-(1 << 62), 1 << 62, ns, dtype=np.int64)
        exp = oracle.chained_join_i64(rk, rp, sk, sp, H=max(1, nr // 8))
    else:
        rk, sk = (a.astype(np.int32) for a in _fuzz_keys(rng, lo, span, nr, ns))
        rp = sp = None
        exp = oracle.chained_join_i32(rk, sk, H=max(1, nr // 8))
    o = run(hj, rk, rp, sk, sp, bits)
    assert len(o[0]) == len(exp[0])
    assert oracle.same_multiset(*o, *exp)
    if i % 4 == 0:   # the same inputs through the global (one HBM table) strategy
        hj.set_strategy("global")
        try:
            g_r, g_s = hj.join(dev(rk), None if rp is None else dev(rp), dev(sk), None if sp is None else dev(sp))
            assert hj.strategy_used == "global"
            torch.cuda.synchronize()
        finally:
            hj.set_strategy("auto")
        assert oracle.same_multiset(g_r.cpu().numpy().astype(np.int64), g_s.cpu().numpy().astype(np.int64), *exp)


@pytest.mark.parametrize("wide", [True, False])
@pytest.mark.parametrize("dups", [False, True])
def test_radix_duplicates_in_unprobed_partitions(hj, oracle, wide, dups):
    """has_duplicates() after a join whose probe side reaches only a handful
    of the 4096 build partitions: the on-demand check (radix_detect) covers
    the whole build side, so a repeated build key in a partition no probe row
    reached is still reported, and unique keys are not."""
    n = 200000
    rng = np.random.default_rng(4242 + (1 if wide else 0))
    rk = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=n, replace=False)
    sk = rk[:8].copy()   # 8 probe rows: at most 8 of the 4096 partitions probed
    if dups:
        rk[n - 1] = rk[n - 2]   # (neither key is probed)
    rp = np.arange(n, dtype=np.int64) * 7 + 3
    sp = np.arange(len(sk), dtype=np.int64) + 11
    if wide:
        o = run(hj, rk, rp, sk, sp, 12)
        assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=1000))
    else:
        o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 12)
        ex = oracle.chained_join_i32(rk.astype(np.int32), sk.astype(np.int32), H=1000)
        assert oracle.same_multiset(*o, ex[0].astype(np.int64), ex[1].astype(np.int64))
    assert len(o[0]) == 8
    assert hj.has_duplicates() == dups


@pytest.mark.parametrize("wide", [True, False])
@pytest.mark.parametrize("dups", [False, True])
def test_radix_duplicates_across_build_rounds(hj, oracle, wide, dups):
    """has_duplicates() when the only repeated build key sits in a partition
    too large for one LDS table (2 radix bits: ~10k rows per partition,
    deferred to k_join's list mode, built in rounds of 2560 rows) with its two
    copies in different rounds: the detect path's self-join count
    finds it; unique keys stay unique."""
    n = 40000
    rng = np.random.default_rng(777 + (1 if wide else 0))
    rk = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=n, replace=False)
    if dups:
        rk[n - 1] = rk[0]   # first and last build row: read in different rounds
    sk = rk[1:9].copy()     # 8 probe rows, none with the repeated key
    rp = np.arange(n, dtype=np.int64) * 3 + 1
    sp = np.arange(len(sk), dtype=np.int64) + 5
    if wide:
        o = run(hj, rk, rp, sk, sp, 2)
        assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=1000))
    else:
        o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 2)
        ex = oracle.chained_join_i32(rk.astype(np.int32), sk.astype(np.int32), H=1000)
        assert oracle.same_multiset(*o, ex[0].astype(np.int64), ex[1].astype(np.int64))
    assert len(o[0]) == 8
    assert hj.has_duplicates() == dups


@pytest.mark.parametrize("wide", [True, False])
def test_radix_has_duplicates_hot_key_in_oversized_partition(hj, oracle, wide):
    """has_duplicates() over a build side whose one key repeats 2^17 times in
    partitions far too large for an LDS table (2 radix bits, ~2^18 rows each,
    deferred to k_join's rounds): the rounds' own build flags the repeat and
    radix_detect's count-only self-join of the deferred partitions is then
    skipped (run, it would walk every copy's chain past ~2560
    copies per round, ~m^2 steps) -- correct, and answered in well under a
    second."""
    import time
    n, hot = 1 << 20, 1 << 17
    rng = np.random.default_rng(4242 + (1 if wide else 0))
    rk = rng.choice(np.arange(1, 1 << 30, dtype=np.int64), size=n, replace=False)
    rk[rng.choice(n, size=hot, replace=False)] = 7
    sk = rk[rk != 7][:8].copy()     # 8 probe rows, none with the hot key
    rp = np.arange(n, dtype=np.int64) * 3 + 1
    sp = np.arange(len(sk), dtype=np.int64) + 5
    if wide:
        o = run(hj, rk, rp, sk, sp, 2)
        assert oracle.same_multiset(*o, *oracle.nested_loop_i64(rk, rp, sk, sp))
    else:
        o = run(hj, rk.astype(np.int32), None, sk.astype(np.int32), None, 2)
        assert len(o[0]) == 8 and np.array_equal(np.sort(sk.astype(np.int64)), np.sort(rk[o[0]]))
    assert len(o[0]) == 8
    t0 = time.perf_counter()
    assert hj.has_duplicates()
    assert time.perf_counter() - t0 < 5.0



def test_auto_probe_threshold_by_build_size(hj):
    """AUTO's probe-time choice for a [2^18, 2^21)-row build: from 2^22 probe
    rows on the radix join when the build side has >= 2^20 rows (2^24
    below that) -- same pairs as a forced-global join."""
    nr, ns = 1 << 20, 1 << 22
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EEF, nr, ns, 0.9)
    hj.set_strategy("auto")
    try:
        o_r, o_s = hj.join(rk, rp, sk, sp)
        assert hj.strategy_used == "radix"
        small_r, small_s = hj.join(rk, rp, sk[:ns // 2], sp[:ns // 2])
        assert hj.strategy_used == "global"
        hj.set_strategy("global")
        g_r, g_s = hj.join(rk, rp, sk, sp)
        assert o_r.numel() == g_r.numel()
        order, gorder = torch.argsort(o_s), torch.argsort(g_s)
        assert torch.equal(o_r[order], g_r[gorder]) and torch.equal(o_s[order], g_s[gorder])
    finally:
        hj.set_strategy("auto")
