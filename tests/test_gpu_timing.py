"""Accumulated phase timing (hj_ctx_timing_accumulate / hj_ctx_timing_totals):
build + probe steps run back to back with no host synchronisation between
them (bench.py's timed loop) and the totals still cover every step, past the
64-set event ring."""
import pytest
import torch

from hashjoin import HashJoin

pytestmark = pytest.mark.gpu


def _pkfk(n_r, n_s, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rk = torch.randperm(n_r, device="cuda", generator=g).to(torch.int64)
    rp = torch.arange(n_r, device="cuda", dtype=torch.int64)
    sk = torch.randint(0, n_r, (n_s,), device="cuda", generator=g, dtype=torch.int64)
    sp = torch.arange(n_s, device="cuda", dtype=torch.int64)
    return rk, rp, sk, sp


@pytest.mark.parametrize("steps", [5, 70])
def test_accumulated_timing_covers_every_step(steps):
    n_r, n_s = 1 << 20, 1 << 21
    rk, rp, sk, sp = _pkfk(n_r, n_s, 11)
    hj = HashJoin(0)
    try:
        hj.set_strategy("radix")
        hj.allocate_hash_table(n_r, 64)
        hj.reserve_probe(n_s, 64)
        out_r = torch.empty(n_s, dtype=torch.int64, device="cuda")
        out_s = torch.empty_like(out_r)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        hj.accumulate_timing(True)
        for _ in range(steps):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        tot = hj.timing_totals()
        assert tot["steps"] == steps
        assert tot["build"] > 0 and tot["probe"] > 0 and tot["init"] >= 0
        # the probe's split adds up to the probe phase (same events)
        assert abs(tot["probe_partition"] + tot["probe_join"] - tot["probe"]) <= 1e-3 * tot["probe"] + 1e-3
        # every step joined all of S (PK-FK): the last step's rows are right
        m = int(cnt.item())
        assert m == n_s
        assert bool((rk[out_r[:m]] == sk[out_s[:m]]).all())
        # the totals start again after a read
        again = hj.timing_totals()
        assert again["steps"] == 0 and again["probe"] == 0
        # one more step, then the per-step reading agrees with the totals' scale
        hj.build_table(rk, rp)
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        one = hj.timing_totals()
        assert one["steps"] == 1
        assert 0.2 < one["probe"] / (tot["probe"] / steps) < 5.0
    finally:
        hj.close()


def test_timing_totals_need_accumulating_mode():
    hj = HashJoin(0)
    try:
        hj.set_timing(True)
        with pytest.raises(Exception):
            hj.timing_totals()
        hj.accumulate_timing(True)
        assert hj.timing_totals()["steps"] == 0
        hj.accumulate_timing(False)
        with pytest.raises(Exception):
            hj.timing_totals()
    finally:
        hj.close()
