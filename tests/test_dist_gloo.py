"""World-size-2 gloo tests of the multi-GPU routing + exchange (CPU).

The device kernels cannot run here, so each rank partitions its slice with
the numpy restatement of the routing hash (itself checked against the
library's hj_partition_of in test_abi.py), exchanges through the product's
hashjoin.dist.exchange (the same torch.distributed all-to-all code that runs
over RCCL on the GPU box), joins locally with the oracle, and rank 0 checks
that the union of the per-rank results is exactly the global join."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _route(keys, pays, P):
    from test_abi import _np_partition_of
    pid = _np_partition_of(keys, P)
    order = np.argsort(pid, kind="stable")
    tuples = np.stack([keys[order], pays[order]], axis=1)
    counts = np.bincount(pid, minlength=P).astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(tuples)), torch.from_numpy(counts)


def _worker(rank, world, port, case, outdir):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mlir-hashjoin_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)
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
