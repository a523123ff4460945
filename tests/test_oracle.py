"""CPU tests: the oracle against the golden fixtures and the reference's own
check() (shared_stuff/shared.cpp:129-172, compiled into oracle/_ref/)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases


@pytest.mark.parametrize("case", golden_cases(32))
def test_golden_i32(oracle, case):
    r, s, exp, H = case["r"], case["s"], case["expected"], int(case["H"][0])
    for variant in (1, 2):
        o = oracle.chained_join_i32(r, s, H=H, variant=variant)
        assert np.array_equal(oracle.sorted_pairs(*o), exp)
    nl = oracle.nested_loop_i32(r, s)
    assert np.array_equal(oracle.sorted_pairs(*nl), exp)
    # a different table size H must not change the join (only chain shape)
    o = oracle.chained_join_i32(r, s, H=max(1, len(r)), variant=2)
    assert np.array_equal(oracle.sorted_pairs(*o), exp)


@pytest.mark.parametrize("case", golden_cases(64))
def test_golden_i64(oracle, case):
    rk, rp, sk, sp, exp = case["rk"], case["rp"], case["sk"], case["sp"], case["expected"]
    H = int(case["H"][0])
    for variant in (1, 2):
        o = oracle.chained_join_i64(rk, rp, sk, sp, H=H, variant=variant)
        assert np.array_equal(oracle.sorted_pairs(*o), exp)
    m, _ = oracle.chained_join_i64_omp(rk, rp, sk, sp, H, 2, count_only=True)
    assert m == len(exp)


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "shared.so")),
                    reason="reference harness not built")
@pytest.mark.parametrize("case", golden_cases(32))
def test_golden_pinned_by_reference_check(oracle, case):
    exp = case["expected"]
    assert oracle.ref_check(case["r"], case["s"], exp[:, 0], exp[:, 1]) == 1


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "shared.so")),
                    reason="reference harness not built")
@pytest.mark.parametrize("seed", range(12))
def test_restatement_vs_reference_check(oracle, seed):
    rng = np.random.default_rng(seed)
    nr, ns = int(rng.integers(0, 600)), int(rng.integers(0, 600))
    hi = int(rng.choice([3, 50, 1000, 1 << 30]))
    r = rng.integers(-hi, hi, nr, dtype=np.int64).astype(np.int32)
    s = rng.integers(-hi, hi, ns, dtype=np.int64).astype(np.int32)
    H = int(rng.integers(1, 300))
    o_r, o_s = oracle.chained_join_i32(r, s, H=H, variant=2)
    assert oracle.ref_check(r, s, o_r, o_s) == 1
    if len(o_r):
        assert oracle.ref_check(r, s, o_r[:-1], o_s[:-1]) == -1


def test_reference_check_false_positive_documented(oracle):
    """check() accepts a candidate padded with (0,0) rows when
    R[0] == S[0] is not required -- it sizes its truth vector to the
    candidate.  Our parity therefore compares the exact count first."""
    if not oracle.ref_available():
        pytest.skip("reference harness not built")
    r = np.array([5, 6], np.int32); s = np.array([6, 9], np.int32)
    o_r, o_s = oracle.nested_loop_i32(r, s)
    pad_r = np.concatenate([o_r, [0]]).astype(np.int32)
    pad_s = np.concatenate([o_s, [0]]).astype(np.int32)
    assert oracle.ref_check(r, s, pad_r, pad_s) == 1          # the false positive
    assert not oracle.same_multiset(pad_r, pad_s, o_r, o_s)  # ours rejects it


def test_nested_loop_kat(oracle):
    with np.load(os.path.join(GOLDEN, "nested_loop_kat.npz"), allow_pickle=False) as z:
        t1, t2, rows = z["t1"], z["t2"], z["rows"]
    assert np.array_equal(oracle.nested_init_i32(20, 3), t1)
    assert np.array_equal(oracle.nested_join_rows_i32(t1, t2), rows)
    # outer = larger table: swap sizes and the other table becomes x
    big = oracle.nested_init_i32(30, 2)
    out = oracle.nested_join_rows_i32(t1, big)
    assert out.shape == (20, 2 + 3 - 1)
    assert np.array_equal(out[:, 0], np.arange(20))


def test_pkfk_generator_contract(oracle):
    for frac in (1.0, 0.5, 0.0):
        rk, rp, sk, sp = oracle.gen_pkfk_i64(7, 500, 800, frac)
        assert len(np.unique(rk)) == 500
        er, es = oracle.pkfk_expected(7, 500, 800, frac)
        o = oracle.chained_join_i64(rk, rp, sk, sp)
        assert oracle.same_multiset(*o, er, es)
        if frac == 1.0:
            assert len(er) == 800
    # slices of the global relation equal the whole
    a = oracle.gen_pkfk_i64(9, 1000, 1000)
    b = oracle.gen_pkfk_i64(9, 1000, 1000, r0=250, nr=300, s0=600, ns=400)
    assert np.array_equal(a[0][250:550], b[0]) and np.array_equal(a[2][600:1000], b[2])


def test_omp_baseline_matches(oracle):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(3, 5000, 7000, 0.9)
    m, ph = oracle.chained_join_i64_omp(rk, rp, sk, sp, 5000, 4)
    assert m == len(oracle.pkfk_expected(3, 5000, 7000, 0.9)[0])
    assert (ph >= 0).all()


def test_pair_digest_order_independent(oracle):
    rng = np.random.default_rng(1)
    r = rng.integers(0, 1 << 40, 1000); s = rng.integers(0, 1 << 40, 1000)
    p = rng.permutation(1000)
    assert oracle.pair_digest(r, s) == oracle.pair_digest(r[p], s[p])
    assert oracle.pair_digest(r, s) != oracle.pair_digest(s, r)


def test_selection_kat(oracle):
    """selection.mlir @main: arr[i] = i (128), keep arr[i] < 80.0 -> 0..79."""
    with np.load(os.path.join(GOLDEN, "selection_kat.npz"), allow_pickle=False) as z:
        a, c, vals, rows = z["input"], float(z["value"]), z["values"], z["rows"]
    assert np.array_equal(a, oracle.selection_init_f32(128))
    v, r = oracle.select(a, "lt", c)
    assert np.array_equal(v, vals) and np.array_equal(r, rows)


def test_selection_semantics(oracle):
    """Ordered float compares (NaN never selected); every op against numpy."""
    rng = np.random.default_rng(3)
    a = rng.normal(size=5000).astype(np.float32)
    a[::17] = np.nan; a[::29] = np.inf; a[::31] = -np.inf; a[::37] = 0.25
    ops = {"lt": np.less, "le": np.less_equal, "gt": np.greater, "ge": np.greater_equal, "eq": np.equal}
    for op, f in ops.items():
        v, r = oracle.select(a, op, 0.25)
        keep = np.nonzero(f(a, np.float32(0.25)))[0]
        assert np.array_equal(r, keep) and np.array_equal(v, a[keep])
    v, r = oracle.select(a, "ne", 0.25)
    keep = np.nonzero((a < 0.25) | (a > 0.25))[0]   # ordered: NaN excluded
    assert np.array_equal(r, keep)
    k = rng.integers(-50, 50, 3000)
    for op, f in list(ops.items()) + [("ne", np.not_equal)]:
        v, r = oracle.select(k, op, 7)
        assert np.array_equal(r, np.nonzero(f(k, 7))[0])
