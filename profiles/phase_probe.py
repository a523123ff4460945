#!/usr/bin/env python3
"""Diagnostic: per-phase HIP-event times of the radix join at C3 scale,
probe with writes vs count-only (isolates the output write + cursor atomic)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))
import torch
import hashjoin

lg = int(os.environ.get("LG", "28"))
n = 1 << lg
rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
hj = hashjoin.HashJoin(0)
hj.set_strategy(os.environ.get("STRAT", "radix"))
hj.set_timing(True)
out_r = torch.empty(n, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
res = {}
for it in range(4):
    hj.build_table(rk, rp)
    hj.probe_relation(sk, sp, out_r, out_s)
    t = hj.last_timing()
    hj.count_rows(sk, sync=False)
    tc = hj.last_timing()
    if it >= 1:
        for k, v in t.items(): res.setdefault("probe:" + k, []).append(v)
        res.setdefault("count:probe_join", []).append(tc["probe_join"])
print(json.dumps({k: round(sum(v) / len(v), 3) for k, v in res.items()}))
