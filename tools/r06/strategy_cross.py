"""Global table vs radix join around AUTO's threshold (kRadixMinRows = 2^21
build rows): eager build + probe ms per step, PK-FK, |S| = |R| and 4 |R|."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402

for lg in (19, 20, 21, 22):
    for mult in (1, 4):
        nr, ns = 1 << lg, (1 << lg) * mult
        rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, nr, ns, 1.0)
        out_r = torch.empty(ns, dtype=torch.int64, device="cuda")
        out_s = torch.empty_like(out_r)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        res = {}
        for strat in ("global", "radix", "auto"):
            hj = hashjoin.HashJoin(0)
            hj.set_strategy(strat)
            hj.probe_hint(ns)
            hj.allocate_hash_table(nr, 64)
            hj.build_table(rk, rp)
            hj.reserve_probe(ns, 64)
            for _ in range(5):
                hj.build_table(rk, rp)
                hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                hj.build_table(rk, rp)
                hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
            torch.cuda.synchronize()
            res[strat] = (time.perf_counter() - t0) / 50 * 1e3
            assert int(cnt.item()) == ns
            used = hj.strategy_used
            hj.close()
        print(f"|R|=2^{lg} |S|={mult}x: global {res['global']:.4f}  radix {res['radix']:.4f}  auto {res['auto']:.4f} ms "
              f"(auto used {used})", flush=True)
