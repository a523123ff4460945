"""Multi-GPU hash join: radix routing + RCCL all-to-all over xGMI.

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
The reference is single-GPU (projectDescription.md:23-25 lists "Partitioned
Hash-Join" and "Joining skewed data" as left out); north_star adds this path
(SURVEY 8(e)):

  SHUFFLE (large build sides)
  1. every rank radix-partitions its slice of R and of S by the owner hash
     (hj_dev_partition_*: one HIP histogram + scatter pass each).  FOLDED
     (hj_route_plan > 0: a power-of-two world and a radix-sized local build):
     the owner and the receiver's first radix-pass bin are the top bits of
     the join's own key hash (hj_dev_route_i64), so every rank receives its
     rows already first-pass partitioned and builds / probes with one local
     pass (hj_dev_build_routed_i64 / hj_dev_probe_routed_i64) instead of two,
  2. per relation, one all-to-all of the per-owner counts (world int64),
  3. per relation, one batched group of point-to-point messages (RCCL
     grouped send/recv) of packed 16-B {key, payload} tuples, started
     asynchronously: R's transfer overlaps S's routing, S's overlaps R's build,
  4. local build + probe on the received tuples (hj_dev_*_tuples_i64).
     The output stays distributed: rank p holds the pairs whose key it owns.

  REPLICATE (small build sides, |R| <= replicate_max_rows, SURVEY 8(e) "Small
  R (C2-like)"): R's slices are all-gathered (one RCCL all-gather of at most
  2^21 x 16 B = 32 MiB), every rank builds the whole R and probes its own S
  slice in place -- S never crosses xGMI.  Rank p holds the pairs of its own
  S rows.

`exchange` / `distributed_join` are device-agnostic torch.distributed code:
`hj` is anything with the HashJoin methods partition / build_tuples /
probe_tuples, so the routing, exchange and replication logic runs with gloo
on CPU tensors in tests/ (with the CPU oracle standing in for the kernels).
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

_DEBUG = os.environ.get("HJ_DEBUG") == "1"

# Build sides up to this many rows (global) are replicated instead of routed
# (32 MiB of tuples: one all-gather is cheaper than shuffling S).
REPLICATE_MAX_ROWS = 1 << 21


def _dbg(*a):
    if _DEBUG:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        print(f"[hj.dist {time.time():.3f} rank {dist.get_rank()}]", *a, file=sys.stderr, flush=True)


# Largest slice one rank hands one peer in one collective round.  RCCL moves
# each point-to-point message with a 32-bit byte count internally on some
# paths, so a 4 GiB slice (2^28 16-B tuples) is silently truncated; rounds of
# at most 2^26 rows (1 GiB) stay well clear of that and are still large enough
# to run xGMI at link rate.
MAX_ROWS_PER_ROUND = 1 << 26


def _all_to_all_rows(recv, send, out_rows, in_rows, group, max_rows, self_p2p=False, in_off=None):
    """recv[rows from p] <- every p's send[rows for me]: one batched group of
    point-to-point messages of at most max_rows rows each (views, no staging
    copies).  Sender and receiver cut a slice into the same pieces because
    in_rows on p and out_rows here describe the same slice.  The slice a rank
    keeps is copied locally unless self_p2p (tests: it then goes through the
    backend like any other slice, cut into the same pieces).  in_off: where
    each destination's rows start in send (default: packed in rank order).
    Returns the outstanding works (wait on them before reading recv)."""
    world = len(in_rows)
    me = dist.get_rank(group)
    if in_off is None:
        in_off = [sum(in_rows[:p]) for p in range(world)]
    out_off = [sum(out_rows[:p]) for p in range(world)]
    ops = []
    if self_p2p:
        gme = dist.get_global_rank(group, me) if group is not None else me
        for a in range(0, in_rows[me], max_rows):
            b = min(in_rows[me], a + max_rows)
            ops.append(dist.P2POp(dist.isend, send[in_off[me] + a:in_off[me] + b], gme, group))
            ops.append(dist.P2POp(dist.irecv, recv[out_off[me] + a:out_off[me] + b], gme, group))
    else:
        recv[out_off[me]:out_off[me] + out_rows[me]].copy_(send[in_off[me]:in_off[me] + in_rows[me]])
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
    current stream after the transfer; `recv` is valid from then on.

    parts > 1: every rank's slice moves as `parts` consecutive batches (part
    k = rows [n k / parts, n (k + 1) / parts) of each slice, the same cut on
    both ends), and recv holds part 0's rows from every rank, then part 1's,
    ...: `wait_part(k)` returns part k as soon as it has arrived, so the
    caller can work on it while the later parts are still on the links."""

    def __init__(self, send, counts, group=None, max_rows=None, self_p2p=False, parts=1):
        world = dist.get_world_size(group)
        if counts.numel() != world:
            raise ValueError("one count per rank required")
        max_rows = MAX_ROWS_PER_ROUND if max_rows is None else int(max_rows)
        if max_rows < 1:
            raise ValueError("max_rows must be positive")
        parts = int(parts)
        if parts < 1:
            raise ValueError("parts must be positive")
        counts = counts.contiguous()
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=group)
        host = torch.stack([counts, recv_counts]).cpu()
        self.in_rows, self.out_rows = host[0].tolist(), host[1].tolist()
        self.send = send   # kept alive until the transfer is done
        if world == 1 and not self_p2p:
            # a one-rank shuffle is the identity: the routed rows ARE the
            # received rows (no 2 x 4 GiB self-copy at C3, ~3 ms)
            self.recv = send[:self.out_rows[0]]
            self._parts = [[self.recv[self.out_rows[0] * k // parts:self.out_rows[0] * (k + 1) // parts], []]
                           for k in range(parts)]
            return
        self.recv = torch.empty((sum(self.out_rows), 2), dtype=torch.int64, device=send.device)
        in_off = [sum(self.in_rows[:p]) for p in range(world)]
        cut = lambda n, k: n * k // parts  # noqa: E731
        self._parts = []
        base = 0
        for k in range(parts):
            in_k = [cut(n, k + 1) - cut(n, k) for n in self.in_rows]
            out_k = [cut(n, k + 1) - cut(n, k) for n in self.out_rows]
            off_k = [in_off[p] + cut(self.in_rows[p], k) for p in range(world)]
            recv_k = self.recv[base:base + sum(out_k)]
            base += sum(out_k)
            works = _all_to_all_rows(recv_k, send, out_k, in_k, group, max_rows, self_p2p, in_off=off_k)
            self._parts.append([recv_k, works])

    @property
    def parts(self):
        return len(self._parts)

    def wait_part(self, k):
        for w in self._parts[k][1]:
            w.wait()
        self._parts[k][1] = []
        return self._parts[k][0]

    def wait(self):
        for k in range(len(self._parts)):
            self.wait_part(k)
        return self.recv


class RoutedExchange:
    """The folded routing's transfer.  send holds, destination by destination,
    that destination's bins 0 .. F-1 in order; counts (world * F) their sizes.
    The bin counts are exchanged (one all-to-all of world * F int64), then the
    rows move in `parts` batches: part k = bins [bounds[k], bounds[k + 1]) of
    every source, source by source -- whole first-pass segments, so part k can
    be partitioned and joined as soon as it has arrived.  part_counts[k]
    (device, nsrc x bins) describes part k's layout for the routed build /
    probe."""

    def __init__(self, send, counts, nbins, group=None, max_rows=None, self_p2p=False, parts=1):
        world = dist.get_world_size(group)
        if counts.numel() != world * nbins:
            raise ValueError("one count per (rank, bin) required")
        max_rows = MAX_ROWS_PER_ROUND if max_rows is None else int(max_rows)
        parts = max(1, min(int(parts), nbins))
        counts = counts.contiguous().view(world, nbins)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=group)
        host = torch.stack([counts, recv_counts]).cpu()
        send_c, recv_c = host[0], host[1]
        self.send = send
        self.bounds = [nbins * k // parts for k in range(parts + 1)]
        self.in_rows = send_c.sum(1).tolist()
        self.out_rows = recv_c.sum(1).tolist()
        dest_off = [int(send_c[:d].sum()) for d in range(world)]
        self.part_counts = []
        self._parts = []
        alias = world == 1 and not self_p2p
        self.recv = send[:self.out_rows[0]] if alias else torch.empty((sum(self.out_rows), 2), dtype=torch.int64,
                                                                         device=send.device)
        base = 0
        for k in range(parts):
            b0, b1 = self.bounds[k], self.bounds[k + 1]
            in_k = send_c[:, b0:b1].sum(1).tolist()
            out_k = recv_c[:, b0:b1].sum(1).tolist()
            off_k = [dest_off[d] + int(send_c[d, :b0].sum()) for d in range(world)]
            recv_k = self.recv[base:base + sum(out_k)]
            base += sum(out_k)
            works = [] if alias else _all_to_all_rows(recv_k, send, out_k, in_k, group, max_rows, self_p2p,
                                                      in_off=off_k)
            self._parts.append([recv_k, works])
            self.part_counts.append(recv_counts[:, b0:b1].contiguous())

    @property
    def parts(self):
        return len(self._parts)

    def wait_part(self, k):
        for w in self._parts[k][1]:
            w.wait()
        self._parts[k][1] = []
        return self._parts[k][0]

    def wait(self):
        for k in range(len(self._parts)):
            self.wait_part(k)
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


def all_gather_rows(tuples, group=None):
    """Every rank's (n_p, 2) int64 tuples, concatenated in rank order, on
    every rank: counts all-gathered first, slices padded to the largest one
    for one all_gather_into_tensor (RCCL all-gather), then compacted."""
    world = dist.get_world_size(group)
    n = torch.tensor([tuples.shape[0]], dtype=torch.int64, device=tuples.device)
    ns = torch.empty(world, dtype=torch.int64, device=tuples.device)
    dist.all_gather_into_tensor(ns, n, group=group)
    counts = ns.cpu().tolist()
    mx = max(counts) if counts else 0
    if mx == 0:
        return torch.empty((0, 2), dtype=torch.int64, device=tuples.device)
    pad = torch.zeros((mx, 2), dtype=torch.int64, device=tuples.device)
    pad[:tuples.shape[0]].copy_(tuples)
    full = torch.empty((world * mx, 2), dtype=torch.int64, device=tuples.device)
    dist.all_gather_into_tensor(full, pad, group=group)
    return torch.cat([full[p * mx:p * mx + counts[p]] for p in range(world)])


def _checked_count(cnt):
    """The match count a probe returned; bit 63 set (a negative int64) means
    an internal work list overflowed and the pairs are incomplete (hj.h), so
    it is an error, never a row count (as in HashJoin.join)."""
    m = int(cnt.item())
    if m < 0:
        raise RuntimeError("hash join: internal work list overflow (count flagged)")
    return m


def _probe_all(hj, tuples, capacity, probe=None):
    """Probe into an output sized optimistically, once more at the exact M.
    probe(tuples, out_r, out_s) -> count tensor (default hj.probe_tuples)."""
    probe = hj.probe_tuples if probe is None else probe
    cap = max(1, tuples.shape[0] if capacity is None else int(capacity))
    for _ in range(2):
        out_r = torch.empty(cap, dtype=torch.int64, device=tuples.device)
        out_s = torch.empty(cap, dtype=torch.int64, device=tuples.device)
        m = _checked_count(probe(tuples, out_r, out_s))
        if m <= cap:
            return out_r[:m], out_s[:m]
        cap = m
    raise RuntimeError("distributed join output did not fit after resizing")


def _probe_parts(hj, parts, capacity, total, device, probes=None):
    """Probe each received part of S as soon as it is there (callables that
    wait for it), into one output sized `capacity` (default: the S rows
    received); a part whose pairs do not fit what is left is probed again
    into a buffer of its own at the exact M and the pieces are joined.
    probes[k](tuples, out_r, out_s) probes part k (default hj.probe_tuples)."""
    cap = max(1, total if capacity is None else int(capacity))
    out_r = torch.empty(cap, dtype=torch.int64, device=device)
    out_s = torch.empty(cap, dtype=torch.int64, device=device)
    pos, extra = 0, []
    for k, get in enumerate(parts):
        probe = hj.probe_tuples if probes is None else probes[k]
        t = get()
        if t.shape[0] == 0:
            continue
        m = None
        if cap > pos:
            m = _checked_count(probe(t, out_r[pos:], out_s[pos:]))
            if m <= cap - pos:
                pos += m
                continue
        extra.append(_probe_all(hj, t, m, probe))   # (the rows written past pos are dropped)
    if not extra:
        return out_r[:pos], out_s[:pos]
    return (torch.cat([out_r[:pos]] + [e[0] for e in extra]), torch.cat([out_s[:pos]] + [e[1] for e in extra]))


# S moves in this many consecutive batches when ranks exchange over links, so
# that the probe of one part overlaps the transfer of the next (a part of
# 2^24 rows probes in ~0.56 ms, about what its 0.25 GiB take on the links at
# N = 8); at world size 1 there is no transfer to hide.
S_PARTS = 2


def distributed_join(hj, rkey, rpay, skey, spay, group=None, capacity=None, phases=None,
                     replicate_max_rows=None, max_rows=None, self_p2p=False, n_build_global=None,
                     s_parts=None, route_bits=None):
    """Join this rank's slices of R and S against every other rank's.

    hj: a hashjoin.HashJoin on this rank's GPU (or any object with its
    partition / build_tuples / probe_tuples methods).  Returns this rank's
    share of the result (out_r, out_s) = (R.pay, S.pay): the pairs of keys it
    owns (shuffle) or of its own S rows (replicate).  `phases`, if a dict,
    receives events (start, s_route, routed, built, probed) for timing (CUDA
    events on GPU tensors, else host timestamps; s_route -> routed is S's
    routing, absent when R is replicated), "rows" = (R rows built, S rows
    probed) and "mode" = "shuffle" | "replicate".  n_build_global: |R| over
    all ranks when the caller knows it (the same value on every rank); it
    saves the all-reduce and host round trip that otherwise decide between
    replicating and shuffling R (~0.15 ms per call).  s_parts: batches the
    shuffled S moves in (default S_PARTS, 1 at world size 1).  route_bits: the
    folded routing's bins per owner (default hj.route_plan's choice; 0 routes
    by owner only and the receivers run both local passes)."""
    if replicate_max_rows is None:
        replicate_max_rows = REPLICATE_MAX_ROWS
    cuda = rkey.is_cuda
    ev = (lambda name: _event(phases, name, cuda)) if phases is not None else (lambda name: None)
    ev("start")
    if n_build_global is None:
        n_r = torch.tensor([rkey.numel()], dtype=torch.int64, device=rkey.device)
        dist.all_reduce(n_r, group=group)
        n_build_global = int(n_r.item())
    if int(n_build_global) <= replicate_max_rows:
        # small build side: every rank builds all of R, S stays where it is
        _dbg("replicate", int(n_build_global), skey.numel())
        mine = torch.stack([rkey, rpay], dim=1).contiguous()
        all_r = all_gather_rows(mine, group)
        local_s = torch.stack([skey, spay], dim=1).contiguous()
        ev("routed")
        hj.build_tuples(all_r)
        ev("built")
        if phases is not None:
            phases["rows"] = (all_r.shape[0], local_s.shape[0])
            phases["mode"] = "replicate"
        out = _probe_all(hj, local_s, capacity)
        ev("probed")
        return out
    world = dist.get_world_size(group)
    if s_parts is None:
        s_parts = S_PARTS if world > 1 else 1
    if route_bits is not None:
        sub = int(route_bits) if (world & (world - 1)) == 0 else 0
    else:
        sub = hj.route_plan(int(n_build_global), world) if hasattr(hj, "route_plan") else 0
    if sub > 0:
        # folded: rows arrive first-pass partitioned (one local pass fewer)
        _dbg("route folded", rkey.numel(), skey.numel(), sub)
        nb = 1 << sub
        send_r, cr = hj.route(rkey, rpay, world, sub, slot="r")
        xr = RoutedExchange(send_r, cr, nb, group, max_rows, self_p2p)
        ev("s_route")   # S's share of the route phase: its first partition pass happens here
        send_s, cs = hj.route(skey, spay, world, sub, slot="s")
        xs = RoutedExchange(send_s, cs, nb, group, max_rows, self_p2p, parts=s_parts)
        ev("routed")
        recv_r = xr.wait()
        hj.build_routed(recv_r, xr.part_counts[0], world, sub)
        ev("built")
        n_s = sum(xs.out_rows)
        if phases is not None:
            phases["rows"] = (recv_r.shape[0], n_s)
            phases["mode"] = "shuffle"
            phases["folded"] = True
        probes = [(lambda t, o_r, o_s, k=k: hj.probe_routed(t, xs.part_counts[k], xs.bounds[k], o_r, o_s))
                  for k in range(xs.parts)]
        out = _probe_parts(hj, [lambda k=k: xs.wait_part(k) for k in range(xs.parts)], capacity, n_s, rkey.device,
                           probes)
        ev("probed")
        return out
    _dbg("route", rkey.numel(), skey.numel())
    send_r, cr = hj.partition(rkey, rpay, world)
    xr = Exchange(send_r, cr, group, max_rows, self_p2p)
    ev("s_route")
    send_s, cs = hj.partition(skey, spay, world)
    xs = Exchange(send_s, cs, group, max_rows, self_p2p, parts=s_parts)
    ev("routed")
    recv_r = xr.wait()
    _dbg("build", recv_r.shape[0])
    hj.build_tuples(recv_r)
    ev("built")
    n_s = sum(xs.out_rows)
    _dbg("probe", n_s, xs.parts)
    if phases is not None:
        phases["rows"] = (recv_r.shape[0], n_s)
        phases["mode"] = "shuffle"
    out = _probe_parts(hj, [lambda k=k: xs.wait_part(k) for k in range(xs.parts)], capacity, n_s, rkey.device)
    ev("probed")
    return out


class _HostMark:
    """Host-clock stand-in for a CUDA event (CPU tensors)."""

    def __init__(self):
        self.t = time.perf_counter()

    def synchronize(self):
        pass

    def elapsed_time(self, other):
        return (other.t - self.t) * 1000.0


def _event(store, name, cuda=True):
    if not cuda:
        e = _HostMark()
    else:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
    store[name] = e
    return e
