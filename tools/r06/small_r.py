"""Small build sides against a large probe side (AUTO -> the global table):
eager build + probe ms per step, PK-FK, |S| = 2^26."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402

ns = 1 << 26
for lg in (10, 11, 12, 14, 16, 18):
    nr = 1 << lg
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, nr, ns, 1.0)
    out_r = torch.empty(ns, dtype=torch.int64, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    res = {}
    for strat in ("auto", "radix"):
        hj = hashjoin.HashJoin(0)
        hj.set_strategy(strat)
        hj.probe_hint(ns)
        hj.allocate_hash_table(nr, 64)
        hj.build_table(rk, rp)
        hj.reserve_probe(ns, 64)
        for _ in range(3):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        res[strat] = ((time.perf_counter() - t0) / 20 * 1e3, hj.strategy_used)
        assert int(cnt.item()) == ns
        hj.close()
    floor = ns * 32 / 6.5e12 * 1e3
    print(f"|R|=2^{lg} |S|=2^26: auto {res['auto'][0]:.4f} ms ({res['auto'][1]}), radix {res['radix'][0]:.4f} ms; "
          f"stream floor (S in + pairs out at 6.5 TB/s) {floor:.3f} ms", flush=True)
