"""World-size-2 gloo tests of the multi-GPU routing + exchange (CPU).

The device kernels cannot run here, so each rank partitions its slice with
the numpy restatement of the routing hash (itself checked against the
library's hj_partition_of in test_abi.py), exchanges through the product's
hashjoin.dist.exchange (the same torch.distributed all-to-all code that runs
over RCCL on the GPU box), joins locally with the oracle, and rank 0 checks
that the union of the per-rank results is exactly the global join."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
# a rank that never reaches its rendezvous must fail the test, not hang the
# suite
pytestmark = pytest.mark.timeout(300, method="thread")


def _rdzv(tmp_path):
    """A per-test FileStore rendezvous: no TCP port is
    probed, closed and re-bound, so no other process can take it between the
    probe and init_process_group."""
    return "file://" + str(tmp_path / "rdzv")


def _init(rank, world, rdzv):
    dist.init_process_group("gloo", init_method=rdzv, rank=rank, world_size=world)


def _route(keys, pays, P):
    from test_abi import _np_partition_of
    pid = _np_partition_of(keys, P)
    order = np.argsort(pid, kind="stable")
    tuples = np.stack([keys[order], pays[order]], axis=1)
    counts = np.bincount(pid, minlength=P).astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(tuples)), torch.from_numpy(counts)


def _worker(rank, world, rdzv, case, outdir):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mlir-hashjoin_amd"))
    _init(rank, world, rdzv)
    from oracle import pyoracle as O
    from hashjoin.dist import exchange
    NR, NS = case["NR"], case["NS"]
    # this rank's slice of the global relations (counter-based generator)
    r0, nr = rank * NR // world, (rank + 1) * NR // world - rank * NR // world
    s0, ns = rank * NS // world, (rank + 1) * NS // world - rank * NS // world
    if case["dist"] == "pkfk":
        rk, rp, sk, sp = O.gen_pkfk_i64(case["seed"], NR, NS, case["frac"], r0, nr, s0, ns)
    else:
        rk, rp = O.gen_uniform_i64(case["seed"], 1, 1, case["hi"], nr, i0=r0)
        sk, sp = O.gen_uniform_i64(case["seed"], 2, 1, case["hi"], ns, i0=s0)
    send_r, cr = _route(rk, rp, world)
    send_s, cs = _route(sk, sp, world)
    recv_r, recv_s, splits = exchange(send_r, cr, send_s, cs, max_rows=case.get("max_rows"))
    assert sum(splits["out_r"]) == recv_r.shape[0]
    # every received row is owned by this rank
    from test_abi import _np_partition_of
    if recv_r.shape[0]:
        assert (_np_partition_of(recv_r[:, 0].numpy(), world) == rank).all()
    if recv_s.shape[0]:
        assert (_np_partition_of(recv_s[:, 0].numpy(), world) == rank).all()
    a = recv_r.numpy(); b = recv_s.numpy()
    o_r, o_s = O.chained_join_i64(a[:, 0], a[:, 1], b[:, 0], b[:, 1], H=max(1, len(a)))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), r=o_r, s=o_s, nr=np.array([len(a)]),
             ns=np.array([len(b)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=11),
    dict(dist="uniform", NR=2000, NS=2500, hi=300, seed=12),      # duplicates both sides
    dict(dist="pkfk", NR=7, NS=3, frac=1.0, seed=13),             # tiny / ragged
    dict(dist="pkfk", NR=3001, NS=4999, frac=0.7, seed=14, max_rows=97),  # slices cut in pieces
    dict(dist="pkfk", NR=4000, NS=6001, frac=0.9, seed=15, max_rows=300, world=3),
    dict(dist="uniform", NR=5000, NS=7001, hi=900, seed=16, max_rows=211, world=4),
], ids=["pkfk", "uniform_dups", "tiny", "pieces", "three_ranks_pieces", "four_ranks_dups_pieces"])
def test_two_rank_exchange_join(case, tmp_path, oracle):
    world = case.get("world", 2)
    mp.spawn(_worker, args=(world, _rdzv(tmp_path), case, str(tmp_path)), nprocs=world, join=True)
    rs, ss, tot_r, tot_s = [], [], 0, 0
    for k in range(world):
        with np.load(tmp_path / f"rank{k}.npz", allow_pickle=False) as z:
            rs.append(z["r"]); ss.append(z["s"]); tot_r += int(z["nr"][0]); tot_s += int(z["ns"][0])
    assert tot_r == case["NR"] and tot_s == case["NS"]      # nothing lost or duplicated in transit
    if case["dist"] == "pkfk":
        er, es = oracle.pkfk_expected(case["seed"], case["NR"], case["NS"], case["frac"])
    else:
        rk, rp = oracle.gen_uniform_i64(case["seed"], 1, 1, case["hi"], case["NR"])
        sk, sp = oracle.gen_uniform_i64(case["seed"], 2, 1, case["hi"], case["NS"])
        er, es = oracle.nested_loop_i64(rk, rp, sk, sp)
    assert oracle.same_multiset(np.concatenate(rs), np.concatenate(ss), er, es)


# ---------------------------------------------------------------------------
# distributed_join itself (routing / replication, capacity retry, pieces) with
# the device kernels replaced by CPU stand-ins: partition = the numpy
# restatement of the routing hash, build/probe = the oracle's join_v2
# restatement.  The composition is the product's hashjoin.dist code.
class _CpuJoin:
    """HashJoin's partition / build_tuples / probe_tuples on CPU tensors."""

    def __init__(self, flag=False, plan=None):
        from oracle import pyoracle as O
        self.O = O
        self.r = None
        self.calls = {"partition": 0, "build": 0, "probe": 0}
        self.flag = flag   # probes return a count with bit 63 set (work list overflowed)
        if plan is not None:   # the library's own folded-routing plan (host function, no GPU)
            self.route_plan = plan

    def partition(self, key, pay, nparts):
        self.calls["partition"] += 1
        return _route(key.numpy(), pay.numpy(), nparts)

    def build_tuples(self, t):
        self.calls["build"] += 1
        self.r = t.numpy().copy()

    # the folded routing (hj_dev_route_i64 / _build_routed / _probe_routed):
    # parts = top log2(nranks) + sub bits of the radix hash key * 0x9E37...15
    @staticmethod
    def _rparts(keys, bits):
        h = keys.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        return (h >> np.uint64(64 - bits)).astype(np.int64)

    def route(self, key, pay, nranks, sub, slot=None):
        self.calls["partition"] += 1
        g = nranks.bit_length() - 1
        k, p = key.numpy(), pay.numpy()
        part = self._rparts(k, g + sub)
        order = np.argsort(part, kind="stable")
        t = np.stack([k[order], p[order]], axis=1)
        return torch.from_numpy(np.ascontiguousarray(t)), torch.from_numpy(
            np.bincount(part, minlength=nranks << sub).astype(np.int64))

    def _check_layout(self, t, counts, bin0, nranks, sub):
        """Rows of source s, bin bin0 + j sit where counts says, and carry
        this rank's owner bits and that bin."""
        g = nranks.bit_length() - 1
        keys = t.numpy()[:, 0]
        part = self._rparts(keys, g + sub)
        c = counts.numpy()
        assert c.sum() == len(keys)
        pos = 0
        for s_ in range(c.shape[0]):
            for j in range(c.shape[1]):
                seg = part[pos:pos + c[s_, j]]
                assert (seg == ((dist.get_rank() << sub) | (bin0 + j))).all()
                pos += c[s_, j]

    def build_routed(self, t, counts, nranks, sub):
        self.calls["build"] += 1
        self._check_layout(t, counts, 0, nranks, sub)
        self.routed = (nranks, sub)
        self.r = t.numpy().copy()

    def probe_routed(self, t, counts, bin0, out_r, out_s):
        self._check_layout(t, counts, bin0, *self.routed)
        return self.probe_tuples(t, out_r, out_s)

    def probe_tuples(self, t, out_r, out_s):
        self.calls["probe"] += 1
        s = t.numpy()
        o_r, o_s = self.O.chained_join_i64(self.r[:, 0], self.r[:, 1], s[:, 0], s[:, 1], H=max(1, len(self.r)))
        m = len(o_r)
        k = min(m, out_r.numel())
        out_r[:k] = torch.from_numpy(o_r[:k])
        out_s[:k] = torch.from_numpy(o_s[:k])
        if self.flag:
            return torch.tensor([m | -(1 << 63)], dtype=torch.int64)
        return torch.tensor([m], dtype=torch.int64)


def _relations(case, rank, world):
    from oracle import pyoracle as O
    NR, NS = case["NR"], case["NS"]
    r0, nr = rank * NR // world, (rank + 1) * NR // world - rank * NR // world
    s0, ns = rank * NS // world, (rank + 1) * NS // world - rank * NS // world
    if case["dist"] == "pkfk":
        return O.gen_pkfk_i64(case["seed"], NR, NS, case["frac"], r0, nr, s0, ns)
    rk, rp = O.gen_uniform_i64(case["seed"], 1, case.get("lo", 1), case["hi"], nr, i0=r0)
    sk, sp = O.gen_uniform_i64(case["seed"], 2, case.get("lo", 1), case["hi"], ns, i0=s0)
    return rk, rp, sk, sp


def _dj_worker(rank, world, rdzv, case, outdir):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mlir-hashjoin_amd"))
    _init(rank, world, rdzv)
    from hashjoin.dist import distributed_join
    from test_abi import _np_partition_of
    rk, rp, sk, sp = (torch.from_numpy(x) for x in _relations(case, rank, world))
    plan = None
    if case.get("plan_n"):
        # the N = 8 product plan: hj_route_plan for the bench's global |R|
        # (2^28 over 8 ranks -> 6 bins per owner), applied to small relations
        import hashjoin
        sub = hashjoin.HashJoin.route_plan(case["plan_n"], world)
        assert sub == case["plan_sub"]
        plan = (lambda n, w: sub)
    hj = _CpuJoin(flag=case.get("flag", False), plan=plan)
    ph = {}
    if case.get("flag"):
        # a count flagged by bit 63 is an error on every probe path, never a
        # (negative) row count
        import pytest as _pt
        with _pt.raises(RuntimeError, match="overflow"):
            distributed_join(hj, rk, rp, sk, sp, capacity=case.get("capacity"), phases=ph,
                             replicate_max_rows=case.get("replicate", 0), route_bits=case.get("route_bits"),
                             s_parts=case.get("s_parts"))
        np.savez(os.path.join(outdir, f"dj{rank}.npz"), r=np.zeros(0, np.int64), s=np.zeros(0, np.int64),
                 nr=np.array([0]), ns=np.array([0]), mode=np.array([False]))
        dist.barrier()
        dist.destroy_process_group()
        return
    o_r, o_s = distributed_join(hj, rk, rp, sk, sp, capacity=case.get("capacity"), phases=ph,
                                replicate_max_rows=case.get("replicate", 0), max_rows=case.get("max_rows"),
                                n_build_global=case["NR"] if case.get("known_nr") else None,
                                s_parts=case.get("s_parts"), route_bits=case.get("route_bits"))
    nrows = ph["rows"]
    if ph["mode"] == "shuffle":
        # every output key is owned here (S.pay of the generators is the global row id)
        assert hj.calls["partition"] == 2
        full_sk = _relations(case, 0, 1)[2]
        if o_s.numel():
            if ph.get("folded"):   # owner = the top log2(world) bits of the radix hash
                own = _CpuJoin._rparts(full_sk[o_s.numpy()], world.bit_length() - 1) if world > 1 else 0
                assert (np.asarray(own) == rank).all()
            else:
                assert (_np_partition_of(full_sk[o_s.numpy()], world) == rank).all()
        folded = (case.get("route_bits") or case.get("plan_sub", 0)) > 0 and (world & (world - 1)) == 0
        assert ph.get("folded", False) == folded
    else:
        assert hj.calls["partition"] == 0 and nrows[0] == case["NR"]
    assert ph["start"].elapsed_time(ph["probed"]) >= 0.0
    np.savez(os.path.join(outdir, f"dj{rank}.npz"), r=o_r.numpy(), s=o_s.numpy(), nr=np.array([nrows[0]]),
             ns=np.array([nrows[1]]), mode=np.array([ph["mode"] == "shuffle"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=21),
    dict(dist="uniform", NR=2000, NS=2500, hi=300, seed=22),                    # duplicates both sides
    dict(dist="uniform", NR=1500, NS=1800, lo=-(1 << 63), hi=-(1 << 63) + 40, seed=23),  # INT64_MIN keys
    dict(dist="pkfk", NR=4000, NS=6001, frac=0.9, seed=24, capacity=1, world=3),  # output resized
    dict(dist="pkfk", NR=3001, NS=4999, frac=0.7, seed=25, max_rows=97),       # slices cut in pieces
    dict(dist="pkfk", NR=700, NS=9000, frac=1.0, seed=26, replicate=1 << 21),  # small R: replicated
    dict(dist="uniform", NR=900, NS=1200, hi=50, seed=27, replicate=1 << 21, world=3, capacity=5),
    dict(dist="pkfk", NR=5, NS=3, frac=1.0, seed=28, world=4),                 # ranks without rows
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=29, known_nr=True),     # |R| given: no all-reduce
    dict(dist="pkfk", NR=700, NS=9000, frac=1.0, seed=30, replicate=1 << 21, known_nr=True, world=3),
    dict(dist="pkfk", NR=3000, NS=5001, frac=0.9, seed=31, s_parts=3, world=3, max_rows=113),  # S in 3 batches
    dict(dist="uniform", NR=2000, NS=2500, hi=200, seed=32, s_parts=4, capacity=1000),  # parts overflow the output
    dict(dist="pkfk", NR=7, NS=2, frac=1.0, seed=33, s_parts=5, world=2),               # empty parts
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=34, world=1),                    # identity exchange
    dict(dist="uniform", NR=2000, NS=2500, hi=300, seed=35, world=1, s_parts=2, capacity=700),
    # the folded routing: rows arrive first-pass partitioned (layout checked per part)
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=36, route_bits=3),
    dict(dist="uniform", NR=2000, NS=2600, hi=300, seed=37, route_bits=2, s_parts=3, world=4, max_rows=101),
    dict(dist="pkfk", NR=4000, NS=6001, frac=0.9, seed=38, route_bits=4, world=3),      # 3 ranks: not folded
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=39, route_bits=5, world=1, s_parts=2, capacity=900),
    # the N = 8 product layout: 8 owners x 2^6 bins (9 routing bits, hj_route_plan's maximum), S in 2 parts
    dict(dist="pkfk", NR=6000, NS=9001, frac=0.9, seed=40, route_bits=6, world=8),
    dict(dist="uniform", NR=4000, NS=5000, hi=700, seed=41, plan_n=1 << 28, plan_sub=6, world=8, s_parts=3,
         max_rows=173),
], ids=["pkfk", "dups", "int64_min", "resize_3ranks", "pieces", "replicate", "replicate_dups_3ranks",
        "tiny_4ranks", "known_build_size", "known_build_size_replicate", "s_parts3", "s_parts_overflow",
        "s_parts_empty", "one_rank", "one_rank_s_parts2", "folded", "folded_4ranks_parts", "folded_3ranks_falls_back",
        "folded_one_rank_parts", "folded_8ranks_sub6", "folded_8ranks_product_plan_dups"])
def test_distributed_join_gloo(case, tmp_path, oracle):
    world = case.get("world", 2)
    mp.spawn(_dj_worker, args=(world, _rdzv(tmp_path), case, str(tmp_path)), nprocs=world, join=True)
    rs, ss = [], []
    for k in range(world):
        with np.load(tmp_path / f"dj{k}.npz", allow_pickle=False) as z:
            rs.append(z["r"]); ss.append(z["s"])
    parts = [_relations(case, k, world) for k in range(world)]
    rk, rp, sk, sp = (np.concatenate([p[i] for p in parts]) for i in range(4))
    er, es = oracle.nested_loop_i64(rk, rp, sk, sp)
    assert oracle.same_multiset(np.concatenate(rs), np.concatenate(ss), er, es)


@pytest.mark.parametrize("case", [
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=50, flag=True),                  # shuffle, one part
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=51, flag=True, s_parts=2),       # shuffle, parts
    dict(dist="pkfk", NR=3000, NS=5000, frac=0.8, seed=52, flag=True, route_bits=3),    # folded
    dict(dist="pkfk", NR=700, NS=900, frac=1.0, seed=53, flag=True, replicate=1 << 21),  # replicate
], ids=["shuffle", "shuffle_parts", "folded", "replicate"])
def test_distributed_join_flagged_count_raises(case, tmp_path):
    """a probe count with bit 63 set (an internal work list
    overflowed) must raise on every distributed path instead of reading as a
    negative M (a silently truncated or empty result)."""
    mp.spawn(_dj_worker, args=(2, _rdzv(tmp_path), case, str(tmp_path)), nprocs=2, join=True)


def test_checked_count_helpers():
    """_probe_all / _probe_parts reject a flagged count (no process group)."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mlir-hashjoin_amd"))
    from hashjoin.dist import _probe_all, _probe_parts
    t = torch.zeros((4, 2), dtype=torch.int64)
    flagged = lambda tt, o_r, o_s: torch.tensor([3 | -(1 << 63)], dtype=torch.int64)
    with pytest.raises(RuntimeError, match="overflow"):
        _probe_all(None, t, 8, flagged)
    with pytest.raises(RuntimeError, match="overflow"):
        _probe_parts(None, [lambda: t], 8, 4, "cpu", [flagged])
    ok = lambda tt, o_r, o_s: torch.tensor([2], dtype=torch.int64)
    o_r, o_s = _probe_all(None, t, 8, ok)
    assert o_r.numel() == 2 and o_s.numel() == 2
