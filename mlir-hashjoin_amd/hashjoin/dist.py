"""Multi-GPU hash join: radix routing + RCCL all-to-all over xGMI.

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
The reference is single-GPU (projectDescription.md:23-24 lists "Partitioned
Hash-Join" as left out); north_star adds this path:

  1. every rank radix-partitions its slice of R and of S by the owner hash
     (hj_dev_partition_*: one HIP histogram + scatter pass each),
  2. per relation, one all-to-all of the per-owner counts (world int64),
  3. per relation, one batched group of point-to-point messages (RCCL
     grouped send/recv) of packed 16-B {key, payload} tuples, started
     asynchronously: R's transfer overlaps S's routing, S's overlaps R's build,
  4. local build + probe on the received tuples (hj_dev_*_tuples_i64).

The output stays distributed: rank p holds the pairs whose key it owns.
`exchange` is device-agnostic torch.distributed code, so the routing and
exchange logic is exercised with gloo on CPU tensors in tests/.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

_DEBUG = os.environ.get("HJ_DEBUG") == "1"


def _dbg(*a):
    if _DEBUG:
        torch.cuda.synchronize()
        print(f"[hj.dist {time.time():.3f} rank {dist.get_rank()}]", *a, file=sys.stderr, flush=True)


# Largest slice one rank hands one peer in one collective round.  RCCL moves
# each point-to-point message with a 32-bit byte count internally on some
# paths, so a 4 GiB slice (2^28 16-B tuples) is silently truncated; rounds of
# at most 2^26 rows (1 GiB) stay well clear of that and are still large enough
# to run xGMI at link rate.
MAX_ROWS_PER_ROUND = 1 << 26


def _all_to_all_rows(recv, send, out_rows, in_rows, group, max_rows):
    """recv[rows from p] <- every p's send[rows for me]: one batched group of
    point-to-point messages of at most max_rows rows each (views, no staging
    copies).  Sender and receiver cut a slice into the same pieces because
    in_rows on p and out_rows here describe the same slice.  Returns the
    outstanding works (wait on them before reading recv)."""
    world = len(in_rows)
    me = dist.get_rank(group)
    in_off = [sum(in_rows[:p]) for p in range(world)]
    out_off = [sum(out_rows[:p]) for p in range(world)]
    recv[out_off[me]:out_off[me] + out_rows[me]].copy_(send[in_off[me]:in_off[me] + in_rows[me]])
    ops = []
    for d in range(1, world):
        # pair ranks by distance so every link carries traffic at once
        to, fr = (me + d) % world, (me - d) % world
        peer_to = dist.get_global_rank(group, to) if group is not None else to
        peer_fr = dist.get_global_rank(group, fr) if group is not None else fr
        for a in range(0, in_rows[to], max_rows):
            b = min(in_rows[to], a + max_rows)
            ops.append(dist.P2POp(dist.isend, send[in_off[to] + a:in_off[to] + b], peer_to, group))
        for a in range(0, out_rows[fr], max_rows):
            b = min(out_rows[fr], a + max_rows)
            ops.append(dist.P2POp(dist.irecv, recv[out_off[fr] + a:out_off[fr] + b], peer_fr, group))
    return dist.batch_isend_irecv(ops) if ops else []


class Exchange:
    """One routed tuple buffer in flight: counts are exchanged at start
    (blocking: they size the receive buffer), the tuples move asynchronously
    (batched point-to-point on the backend's stream).  `wait()` orders the
    current stream after the transfer; `recv` is valid from then on."""

    def __init__(self, send, counts, group=None, max_rows=None):
        world = dist.get_world_size(group)
        if counts.numel() != world:
            raise ValueError("one count per rank required")
        max_rows = MAX_ROWS_PER_ROUND if max_rows is None else int(max_rows)
        if max_rows < 1:
            raise ValueError("max_rows must be positive")
        counts = counts.contiguous()
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=group)
        host = torch.stack([counts, recv_counts]).cpu()
        self.in_rows, self.out_rows = host[0].tolist(), host[1].tolist()
        self.send = send   # kept alive until the transfer is done
        self.recv = torch.empty((sum(self.out_rows), 2), dtype=torch.int64, device=send.device)
        self._works = _all_to_all_rows(self.recv, send, self.out_rows, self.in_rows, group, max_rows)

    def wait(self):
        for w in self._works:
            w.wait()
        self._works = []
        return self.recv


def exchange(send_r, counts_r, send_s, counts_s, group=None, max_rows=None):
    """All-to-all-v of two partitioned tuple buffers.

    send_x: (n, 2) int64 rows grouped by destination rank 0..P-1;
    counts_x: (P,) int64 rows per destination.  Returns (recv_r, recv_s, splits)
    where recv_x holds the rows every rank routed here (grouped by source).
    Slices larger than max_rows (default MAX_ROWS_PER_ROUND) move in pieces."""
    xr = Exchange(send_r, counts_r, group, max_rows)
    xs = Exchange(send_s, counts_s, group, max_rows)
    recv_r, recv_s = xr.wait(), xs.wait()
    return recv_r, recv_s, {"in_r": xr.in_rows, "in_s": xs.in_rows, "out_r": xr.out_rows, "out_s": xs.out_rows}


def distributed_join(hj, rkey, rpay, skey, spay, group=None, capacity=None, phases=None):
    """Join this rank's slices of R and S against every other rank's.

    hj: a hashjoin.HashJoin on this rank's GPU.  Returns this rank's share of
    the result (out_r, out_s) = (R.pay, S.pay) of every pair whose key this
    rank owns.  Transfers overlap compute: R's tuples move while S is routed,
    S's while R is built.  `phases`, if a dict, receives CUDA events
    (start, routed, built, probed) for timing and "rows" = (received R rows,
    received S rows)."""
    world = dist.get_world_size(group)
    ev = (lambda name: _event(phases, name)) if phases is not None else (lambda name: None)
    ev("start")
    _dbg("route", rkey.numel(), skey.numel())
    send_r, cr = hj.partition(rkey, rpay, world)
    xr = Exchange(send_r, cr, group)
    send_s, cs = hj.partition(skey, spay, world)
    xs = Exchange(send_s, cs, group)
    ev("routed")
    recv_r = xr.wait()
    _dbg("build", recv_r.shape[0])
    hj.build_tuples(recv_r)
    ev("built")
    recv_s = xs.wait()
    _dbg("probe", recv_s.shape[0])
    if phases is not None:
        phases["rows"] = (recv_r.shape[0], recv_s.shape[0])
    cap = max(1, recv_s.shape[0] if capacity is None else int(capacity))
    for _ in range(2):
        out_r = torch.empty(cap, dtype=torch.int64, device=recv_s.device)
        out_s = torch.empty(cap, dtype=torch.int64, device=recv_s.device)
        cnt = hj.probe_tuples(recv_s, out_r, out_s)
        ev("probed")
        m = int(cnt.item())
        if m <= cap:
            return out_r[:m], out_s[:m]
        cap = m
    raise RuntimeError("distributed join output did not fit after resizing")


def _event(store, name):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    store[name] = e
    return e
