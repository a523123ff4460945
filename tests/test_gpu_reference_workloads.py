"""The reference's own published workloads (join-performances.md), in its
i32 types (keys i32, payload = row id, output (rowR, rowS) i32):

  REF-A  10M x 10M keys uniform in [1, 100k]  -> ~1e9 result rows (100 matches per probe row)
  REF-B 100M x 100M keys uniform in [1, 1e9]  -> ~1e7 result rows

Too large for the oracle, so size-independent properties pin the result:
per-key pair counts equal cR[k] * cS[k] (so M is exact), every pair is a
true match, and no pair occurs twice.  Together they force the output to be
exactly the nested-loop join of shared.cpp:154-165.
"""
import pytest
import torch

import hashjoin
from hashjoin import HashJoin

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def hj():
    h = HashJoin(0)
    yield h
    h.close()


def _check(r, s, o_r, o_s, kmax):
    m = o_r.numel()
    cr = torch.bincount(r.long(), minlength=kmax + 1)
    cs = torch.bincount(s.long(), minlength=kmax + 1)
    assert m == int((cr * cs).sum().item())
    step = 1 << 27
    per_key = torch.zeros(kmax + 1, dtype=torch.int64, device="cuda")
    for a in range(0, m, step):
        rr = o_r[a:a + step].long()
        ss = o_s[a:a + step].long()
        kr = r[rr]
        assert bool((kr == s[ss]).all())                     # true matches
        per_key += torch.bincount(kr.long(), minlength=kmax + 1)
    assert torch.equal(per_key, cr * cs)                     # each key's pair count
    # no pair twice: (rowS, rowR) pairs are distinct
    key = o_s.long() * r.numel() + o_r.long()
    assert torch.unique(key).numel() == m
    return m


def test_ref_a_10m_dup_heavy(hj):
    n, hi = 10_000_000, 100_000
    r = hashjoin.gen_uniform_i32(0x5EED, 1, 1, hi, n)
    s = hashjoin.gen_uniform_i32(0x5EED, 2, 1, hi, n)
    o_r, o_s = hj.join(r, None, s, None)
    m = _check(r, s, o_r, o_s, hi)
    assert abs(m - 1e9) < 0.01e9


def test_ref_b_100m(hj):
    n, hi = 100_000_000, 1_000_000_000
    r = hashjoin.gen_uniform_i32(0x5EED, 1, 1, hi, n)
    s = hashjoin.gen_uniform_i32(0x5EED, 2, 1, hi, n)
    o_r, o_s = hj.join(r, None, s, None)
    m = o_r.numel()
    rs, _ = torch.sort(r.long())
    exp = int((torch.searchsorted(rs, s.long(), side="right") - torch.searchsorted(rs, s.long())).sum().item())
    assert m == exp and abs(m - 1e7) < 0.01e7
    assert bool((r[o_r.long()] == s[o_s.long()]).all())
    assert torch.unique(o_s.long() * n + o_r.long()).numel() == m
