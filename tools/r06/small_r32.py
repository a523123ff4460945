"""i32 (reference types) small build sides against 2^26 probe rows: the
global table (AUTO below 2^21 build rows), eager build + probe ms."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402

ns = 1 << 26
s = torch.randint(1, 1 << 22, (ns,), dtype=torch.int32, device="cuda")
for lg in (10, 11, 12, 13, 14):
    nr = 1 << lg
    r = torch.randint(1, 1 << 22, (nr,), dtype=torch.int32, device="cuda")
    out_r = torch.empty(ns, dtype=torch.int32, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    hj = hashjoin.HashJoin(0)
    hj.set_strategy("global")
    hj.allocate_hash_table(nr, 32)
    hj.build_table(r)
    for _ in range(3):
        hj.build_table(r)
        hj.probe_relation(s, None, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        hj.build_table(r)
        hj.probe_relation(s, None, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    print(f"i32 |R|=2^{lg} |S|=2^26 global: {ms:.4f} ms, M {int(cnt.item())}", flush=True)
    hj.close()
