"""AUTO build of [2^18, 2^21) rows with and without the probe-size hint:
eager build + probe ms per step (back to back), equal-size PK-FK."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402

for lg in (18, 19, 20):
    n = 1 << lg
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n, 1.0)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for hint in (None, n):
        hj = hashjoin.HashJoin(0)
        hj.probe_hint(hint)
        hj.allocate_hash_table(n, 64)
        hj.build_table(rk, rp)
        hj.reserve_probe(n, 64)
        for _ in range(5):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(100):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 100 * 1e3
        print(f"2^{lg} x 2^{lg} auto, hint {hint}: {ms:.4f} ms/step, plan {hj.radix_plan}, M {int(cnt.item())}",
              flush=True)
        hj.close()
