"""The multi-GPU data path on one GPU.

* distributed_join over RCCL at world size 1, in its own process
  (tests/rccl_worker.py): shuffle with the rank's slice sent through RCCL
  point-to-point in pieces, replicate, repeated and INT64_MIN keys, an
  undersized output, and a >1 GiB self-exchange compared byte for byte.
* the per-owner composition an 8-GPU run executes, on one device: the
  routing kernel splits R and S into P owner slices (hj.partition), each
  owner builds its R slice and probes its S slice (build_tuples /
  probe_tuples); the union must equal the oracle's join (small) or satisfy
  the full-size properties (2^28, P = 8: the C3 split).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import hashjoin
from hashjoin import HashJoin

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hj():
    h = HashJoin(0)
    yield h
    h.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_distributed_join_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_worker.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "RCCL_WORKER_OK" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]


def _owner_join(hj, rk, rp, sk, sp, P):
    """Route R and S onto P owners, join each owner's slices: lists of (o_r, o_s)."""
    tr, cr = hj.partition(rk, rp, P)
    ts, cs = hj.partition(sk, sp, P)
    cr, cs = cr.cpu().tolist(), cs.cpu().tolist()
    offr, offs = np.concatenate([[0], np.cumsum(cr)]), np.concatenate([[0], np.cumsum(cs)])
    outs = []
    for q in range(P):
        hj.build_tuples(tr[offr[q]:offr[q + 1]])
        sq = ts[offs[q]:offs[q + 1]]
        cap = max(1, sq.shape[0])
        for _ in range(2):
            o_r = torch.empty(cap, dtype=torch.int64, device="cuda"); o_s = torch.empty_like(o_r)
            m = int(hj.probe_tuples(sq, o_r, o_s).item())
            if m <= cap:
                break
            cap = m
        outs.append((o_r[:m], o_s[:m], tr[offr[q]:offr[q + 1]], sq))
    return outs


def _owner_join_folded(hj, rk, rp, sk, sp, P, sub, s_parts=1):
    """The folded routing (hj_dev_route_i64): owner and first-pass bin from
    the radix hash; each owner's slices joined with the routed build / probe
    (one local pass), its S in s_parts bin ranges: lists of (o_r, o_s)."""
    F = 1 << sub
    tr, cr = hj.route(rk, rp, P, sub)
    ts, cs = hj.route(sk, sp, P, sub)
    crh, csh = cr.cpu().numpy(), cs.cpu().numpy()
    offr = np.concatenate([[0], np.cumsum(crh)])
    offs = np.concatenate([[0], np.cumsum(csh)])
    outs = []
    for q in range(P):
        hj.build_routed(tr[offr[q * F]:offr[(q + 1) * F]], cr[q * F:(q + 1) * F].view(1, F), P, sub)
        rs, ss = [], []
        for k in range(s_parts):
            b0, b1 = q * F + F * k // s_parts, q * F + F * (k + 1) // s_parts
            sq = ts[offs[b0]:offs[b1]]
            cap = max(1, sq.shape[0])
            for _ in range(2):
                o_r = torch.empty(cap, dtype=torch.int64, device="cuda"); o_s = torch.empty_like(o_r)
                m = int(hj.probe_routed(sq, cs[b0:b1].view(1, b1 - b0), b0 - q * F, o_r, o_s).item())
                if m <= cap:
                    break
                cap = m
            rs.append(o_r[:m]); ss.append(o_s[:m])
        outs.append((torch.cat(rs), torch.cat(ss)))
    return outs


@pytest.mark.parametrize("P,sub,s_parts", [(1, 5, 1), (2, 4, 3), (8, 2, 2), (8, 6, 1)])
@pytest.mark.parametrize("kind", ["pkfk", "dups"])
def test_owner_slices_folded_vs_oracle(hj, oracle, P, sub, s_parts, kind):
    """Folded routing: every owner's slices, routed build + routed probe in bin
    ranges, equal the oracle's join; every slice holds only its owner's keys."""
    if kind == "pkfk":
        rk, rp, sk, sp = oracle.gen_pkfk_i64(70 + P + sub, 40000, 60000, 0.85)
    else:
        rk, rp = oracle.gen_uniform_i64(80 + P + sub, 1, 1, 900, 20000)
        sk, sp = oracle.gen_uniform_i64(80 + P + sub, 2, 1, 900, 25000)
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    outs = _owner_join_folded(hj, d(rk), d(rp), d(sk), d(sp), P, sub, s_parts)
    got_r = np.concatenate([o[0].cpu().numpy() for o in outs])
    got_s = np.concatenate([o[1].cpu().numpy() for o in outs])
    assert oracle.same_multiset(got_r, got_s, *oracle.nested_loop_i64(rk, rp, sk, sp))
    assert hj.join_kernel in ("k_join_b", "k_join_grp")


@pytest.mark.slow
def test_c3_eight_owner_folded_2p28(hj):
    """C3 split over 8 owners by the folded routing (64 first-pass bins per
    owner), each owner built and probed with one local pass."""
    n = 1 << 28
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
    sub = hashjoin.HashJoin.route_plan(n, 8)
    assert sub == 6
    outs = _owner_join_folded(hj, rk, rp, sk, sp, 8, sub, s_parts=2)
    sizes = [o[0].numel() for o in outs]
    assert sum(sizes) == n
    assert max(sizes) / (n / 8) < 1.01
    o_r = torch.cat([o[0] for o in outs])
    o_s = torch.cat([o[1] for o in outs])
    del outs
    assert bool((rk[o_r] == sk[o_s]).all())
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("kind", ["pkfk", "dups"])
def test_owner_slices_vs_oracle(hj, oracle, P, kind):
    from test_abi import _np_partition_of
    if kind == "pkfk":
        rk, rp, sk, sp = oracle.gen_pkfk_i64(50 + P, 40000, 60000, 0.85)
    else:
        rk, rp = oracle.gen_uniform_i64(60 + P, 1, 1, 900, 20000)
        sk, sp = oracle.gen_uniform_i64(60 + P, 2, 1, 900, 25000)
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    outs = _owner_join(hj, d(rk), d(rp), d(sk), d(sp), P)
    got_r = np.concatenate([o[0].cpu().numpy() for o in outs])
    got_s = np.concatenate([o[1].cpu().numpy() for o in outs])
    assert oracle.same_multiset(got_r, got_s, *oracle.nested_loop_i64(rk, rp, sk, sp))
    for q, (_, _, tr, ts) in enumerate(outs):   # every slice holds only its owner's keys
        for t in (tr, ts):
            if t.shape[0]:
                assert (_np_partition_of(t[:, 0].cpu().numpy(), P) == q).all()


@pytest.mark.slow
def test_c3_eight_owner_split_2p28(hj):
    """C3 (2^28 x 2^28 PK-FK) split the way 8 GPUs split it, joined owner by owner."""
    n = 1 << 28
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
    outs = _owner_join(hj, rk, rp, sk, sp, 8)
    sizes = [o[0].numel() for o in outs]
    assert sum(sizes) == n
    assert max(sizes) / (n / 8) < 1.01                      # hash routing: balanced owners
    o_s = torch.cat([o[1] for o in outs])
    o_r = torch.cat([o[0] for o in outs])
    del outs
    assert bool((rk[o_r] == sk[o_s]).all())                  # payloads are global row ids
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))   # every S row once


@pytest.mark.slow
def test_c4_zipf_radix_2p28(hj):
    """C4 at its stated size: Zipf(0.9) probe keys over a 2^28 PK build side."""
    n = 1 << 28
    rk, rp, _, _ = hashjoin.gen_pkfk(0x5EED, n, 0)
    sk, sp = hashjoin.gen_zipf(0x5EED, n, n, 0.9)
    hj.set_strategy("radix")
    try:
        o_r, o_s = hj.join(rk, rp, sk, sp)
    finally:
        hj.set_strategy("auto")
    assert o_r.numel() == n
    assert bool((rk[o_r] == sk[o_s]).all())
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))


@pytest.mark.slow
def test_c4_eight_owner_balance_2p28(hj):
    """The C4 probe side routed onto 8 owners: max/mean within SURVEY 8(e)'s ~1.10."""
    n = 1 << 28
    sk, sp = hashjoin.gen_zipf(0x5EED, n, n, 0.9)
    _, counts = hj.partition(sk, sp, 8)
    c = counts.cpu().numpy().astype(float)
    assert c.sum() == n and c.max() / c.mean() < 1.15


@pytest.mark.slow
def test_c4_eight_owner_balance_folded_2p28(hj):
    """The routing the N = 8 product path takes (folded: owner = the top 3
    bits of the radix hash, hj.route with route_plan(2^28, 8) = 6 bins per
    owner), on the C4 Zipf(0.9) probe side: per-owner rows max/mean < 1.15."""
    n = 1 << 28
    sub = hashjoin.HashJoin.route_plan(n, 8)
    assert sub == 6
    sk, sp = hashjoin.gen_zipf(0x5EED, n, n, 0.9)
    t, counts = hj.route(sk, sp, 8, sub)
    del t
    c = counts.view(8, 1 << sub).sum(dim=1).cpu().numpy().astype(float)
    assert c.sum() == n and c.max() / c.mean() < 1.15


@pytest.mark.slow
def test_c4_eight_owner_folded_2p28(hj):
    """C4 (Zipf(0.9) probe keys over a 2^28 PK build side) split over 8
    owners by the folded routing and joined owner by owner (routed build,
    routed probe in 2 bin ranges): every S row exactly once, every pair a
    true match."""
    n = 1 << 28
    rk, rp, _, _ = hashjoin.gen_pkfk(0x5EED, n, 0)
    sk, sp = hashjoin.gen_zipf(0x5EED, n, n, 0.9)
    sub = hashjoin.HashJoin.route_plan(n, 8)
    outs = _owner_join_folded(hj, rk, rp, sk, sp, 8, sub, s_parts=2)
    assert sum(o[0].numel() for o in outs) == n
    o_r = torch.cat([o[0] for o in outs])
    o_s = torch.cat([o[1] for o in outs])
    del outs
    assert bool((rk[o_r] == sk[o_s]).all())
    assert torch.equal(torch.sort(o_s)[0], torch.arange(n, device="cuda"))


@pytest.mark.parametrize("dups", [False, True])
def test_folded_duplicates_after_parts(hj, oracle, dups):
    """has_duplicates() after a routed build probed in 2 bin ranges: the
    repeat check covers the whole routed build side, not only the bins the
    last hj_dev_probe_routed_i64 call joined.  The repeated key
    is one no probe row meets."""
    rk, rp, sk, sp = oracle.gen_pkfk_i64(91, 40000, 30000, 0.9)
    if dups:
        rk = rk.copy()
        rk[-1] = rk[-2]
        keep = sk != rk[-2]
        sk, sp = sk[keep], sp[keep]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    outs = _owner_join_folded(hj, d(rk), d(rp), d(sk), d(sp), 1, 5, s_parts=2)
    got_r = np.concatenate([o[0].cpu().numpy() for o in outs])
    got_s = np.concatenate([o[1].cpu().numpy() for o in outs])
    assert oracle.same_multiset(got_r, got_s, *oracle.nested_loop_i64(rk, rp, sk, sp))
    assert hj.has_duplicates() == dups
