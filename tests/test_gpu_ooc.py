"""GPU parity of the out-of-core join (hj_host_join_ooc_i64, SURVEY 8(f)
rank 3) against the oracle.  Relations larger than HBM cannot be staged in a
test, so a small device budget forces the same code paths: routing into K
groups through the GPU, per-group builds, and probe sides streamed in many
chunks with copies overlapping the probe."""
import numpy as np
import pytest

from hashjoin import HashJoin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hj():
    h = HashJoin(0)
    yield h
    h.close()


@pytest.mark.parametrize("budget", [0, 1 << 26, 1 << 22, 1 << 20])   # in-core ... 2^20 B: many groups, tiny chunks
def test_pkfk_vs_oracle(hj, oracle, budget):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(31, 300000, 450000, 0.8)
    o_r, o_s = hj.join_host(rk, rp, sk, sp, device_budget=budget)
    assert oracle.same_multiset(o_r, o_s, *oracle.chained_join_i64(rk, rp, sk, sp, H=5000))


def test_duplicates_and_capacity(hj, oracle):
    rk, rp = oracle.gen_uniform_i64(41, 1, 1, 3000, 60000)
    sk, sp = oracle.gen_uniform_i64(41, 2, 1, 3000, 50000)
    exp = oracle.chained_join_i64(rk, rp, sk, sp, H=300)
    assert len(exp[0]) > len(sk)          # more pairs than probe rows: chunk outputs must grow
    o_r, o_s = hj.join_host(rk, rp, sk, sp, device_budget=1 << 21, capacity=10)
    assert oracle.same_multiset(o_r, o_s, *exp)


def test_empty_sides(hj):
    e = np.empty(0, np.int64); k = np.arange(100, dtype=np.int64)
    for a, b in [(e, k), (k, e), (e, e)]:
        o_r, o_s = hj.join_host(a, a, b, b, device_budget=1 << 20)
        assert len(o_r) == 0 and len(o_s) == 0
