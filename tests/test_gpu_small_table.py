"""Global tables small enough to live in LDS (k_probe<..., LDS>, tables of
<= 64 KiB: int64 builds of <= 2048 rows, i32 builds of <= 4096 rows) against
the oracle: unique and repeated build keys, INT64_MIN probe keys (their
tiles take the general path), count-only, i32 reference types, and the sizes
either side of the LDS limit."""
import numpy as np
import pytest
import torch

from hashjoin import HashJoin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hj():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    h = HashJoin(0)
    h.set_strategy("global")
    yield h
    h.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def join(hj, rk, rp, sk, sp):
    if rk.dtype == np.int32:
        o_r, o_s = hj.join(dev(rk), None, dev(sk), None)
    else:
        o_r, o_s = hj.join(dev(rk), dev(rp), dev(sk), dev(sp))
    torch.cuda.synchronize()
    assert hj.strategy_used == "global"
    return o_r.cpu().numpy().astype(np.int64), o_s.cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("nr", [1, 100, 1000, 1024, 2048, 3000])   # 3000: 8192 slots, past the LDS limit
def test_small_table_pkfk(hj, oracle, nr):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(nr, nr, 1 << 20, 0.8)
    o = join(hj, rk, rp, sk, sp)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=max(1, nr // 4)))


def test_small_table_repeated_build_keys(hj, oracle):
    rk, rp = oracle.gen_uniform_i64(61, 1, 1, 300, 1000)
    sk, sp = oracle.gen_uniform_i64(61, 2, 1, 400, 1 << 18)
    o = join(hj, rk, rp, sk, sp)
    assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=100))


def test_small_table_int64_min_probe_keys(hj, oracle):
    I64_MIN = -(1 << 63)
    rk, rp, sk, sp = oracle.gen_pkfk_i64(62, 1500, 1 << 19, 0.9)
    rk[::211] = I64_MIN
    sk[::1777] = I64_MIN
    o = join(hj, rk, rp, sk, sp)
    assert oracle.same_multiset(*o, *oracle.nested_loop_i64(rk, rp, sk[:1 << 19], sp[:1 << 19]))


def test_small_table_count_only(hj, oracle):
    rk, rp, sk, sp = oracle.gen_pkfk_i64(63, 700, 1 << 20, 0.6)
    hj.build_table(dev(rk), dev(rp))
    er, _ = oracle.chained_join_i64(rk, rp, sk, sp, H=100)
    assert hj.count_rows(dev(sk)) == len(er)


@pytest.mark.parametrize("nr", [1000, 4000, 5000])   # i32: 8192 slots x 8 B = 64 KiB; 5000: past it
def test_small_table_i32(hj, oracle, nr):
    r = oracle.gen_uniform_i32(64, 1, 1, 1 << 20, nr)
    s = oracle.gen_uniform_i32(64, 2, 1, 1 << 20, 1 << 20)
    o = join(hj, r, None, s, None)
    assert oracle.same_multiset(*o, *oracle.chained_join_i32(r, s, H=max(1, nr // 4)))


@pytest.mark.parametrize("nr,wide", [(1500, True), (4000, True), (3000, False), (20000, False)])
def test_few_repeated_build_keys(hj, oracle, nr, wide):
    """A handful of repeated build keys: only the tiles whose rows meet one go
    to the general path (every other tile keeps the fast path) -- exact."""
    rng = np.random.default_rng(nr)
    if wide:
        rk, rp = oracle.gen_uniform_i64(nr, 1, 1, 1 << 40, nr)
        rk[nr - 5:] = rk[:5]                      # five keys twice
        sk, sp = oracle.gen_uniform_i64(nr, 2, 1, 1 << 40, 1 << 20)
        idx = rng.integers(0, nr, 1 << 18)
        sk[:1 << 18] = rk[idx]                    # a quarter of S hits R
        sk[rng.integers(0, 1 << 20, 40)] = rk[0]  # forty rows meet a repeated key
        o = join(hj, rk, rp, sk, sp)
        assert oracle.same_multiset(*o, *oracle.chained_join_i64(rk, rp, sk, sp, H=max(1, nr // 4)))
    else:
        r = oracle.gen_uniform_i32(nr, 1, 1, 1 << 30, nr)
        r[nr - 5:] = r[:5]
        s = oracle.gen_uniform_i32(nr, 2, 1, 1 << 30, 1 << 20)
        s[:1 << 18] = r[rng.integers(0, nr, 1 << 18)]
        s[rng.integers(0, 1 << 20, 40)] = r[0]
        o = join(hj, r, None, s, None)
        assert oracle.same_multiset(*o, *oracle.chained_join_i32(r, s, H=max(1, nr // 4)))
