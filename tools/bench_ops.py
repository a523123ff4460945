"""Throughput of the secondary operators: selection and the
nested-loop.mlir row join, on one MI355X, inputs resident in HBM.  One JSON
line per case (HIP-event timing on the current stream, median of 10 after 2
warm-ups); algorithmic bytes as stated in DESIGN.md.

usage: python tools/bench_ops.py  [> profiles/r01_ops_bench.jsonl]
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402
from hashjoin._lib import check, lib  # noqa: E402

HBM = 8000.0


def timed(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    hj = hashjoin.HashJoin(0)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    # selection: 2^28 f32, keep ~50 %
    n = 1 << 28
    x = torch.rand(n, device="cuda", dtype=torch.float32)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    for sel in (0.01, 0.5, 0.99):
        ms = timed(lambda: check(lib.hj_dev_select_f32(hj._ctx, x.data_ptr(), n, 0, sel, out.data_ptr(), None, n,
                                                       cnt.data_ptr(), st), "select"))
        m = int(cnt.item())
        byts = n * 4 * 2 + m * 4   # count pass + write pass read the input; survivors written once
        print(json.dumps({"op": "select_f32 lt", "n": n, "selectivity": round(m / n, 4), "ms": round(ms, 4),
                          "elements_per_s": round(n / ms * 1e3, 1), "algorithmic_GBps": round(byts / ms / 1e6, 1),
                          "frac_hbm": round(byts / ms / 1e6 / HBM, 4)}), flush=True)
    del x, out
    # nested-loop rows: X 2^24 x 4 cols, Y 2^20 x 3 cols, keys in [0, 2^20): ~16 matches... keep PK-FK-like
    rx, ry = 1 << 24, 1 << 20
    X = torch.randint(-(1 << 30), 1 << 30, (rx, 4), dtype=torch.int32, device="cuda")
    Y = torch.randint(-(1 << 30), 1 << 30, (ry, 3), dtype=torch.int32, device="cuda")
    Y[:, 0] = torch.randperm(ry, device="cuda", dtype=torch.int32)   # unique inner keys
    X[:, 0] = torch.randint(0, ry, (rx,), dtype=torch.int32, device="cuda")
    oc = 4 + 3 - 1
    outr = torch.empty((rx, oc), dtype=torch.int32, device="cuda")
    args = (X.data_ptr(), rx, 4, 4, Y.data_ptr(), ry, 3, 3)
    ms = timed(lambda: check(lib.hj_dev_join_rows_i32(hj._ctx, *args, outr.data_ptr(), oc, rx, cnt.data_ptr(), st),
                             "rows"))
    m = int(cnt.item())
    byts = rx * 16 + ry * 12 + m * oc * 4 + m * (16 + 12)   # tables read + rows written + row gathers
    print(json.dumps({"op": "join_rows_i32 (nested-loop.mlir)", "X": [rx, 4], "Y": [ry, 3], "rows": m,
                      "ms": round(ms, 4), "rows_per_s": round(m / ms * 1e3, 1),
                      "algorithmic_GBps": round(byts / ms / 1e6, 1)}), flush=True)
    del X, Y, outr
    # out-of-core: host-resident 2^28 x 2^28 PK-FK, PCIe Gen5 x16 between
    import time
    NR = NS = 1 << 28
    rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, NR, NS)
    h = [t.cpu().numpy() for t in (rk, rp, sk, sp)]
    del rk, rp, sk, sp
    torch.cuda.empty_cache()
    for budget, name in ((0, "R resident, S streamed"), (8 << 30, "8 GiB budget: routed into groups")):
        hj.join_host(*h, device_budget=budget)   # warm-up (page-locking, workspaces)
        t0 = time.perf_counter()
        o_r, o_s = hj.join_host(*h, device_budget=budget)
        dt = time.perf_counter() - t0
        m = len(o_r)
        assert m == NS
        print(json.dumps({"op": "join_host_ooc_i64", "mode": name, "R_rows": NR, "S_rows": NS, "s": round(dt, 4),
                          "probe_tuples_per_s": round(NS / dt, 1),
                          "pcie_bytes_min": (NR + NS) * 16 + m * 16,
                          "pcie_GBps_min": round(((NR + NS) * 16 + m * 16) / dt / 1e9, 1)}), flush=True)
    hj.close()


if __name__ == "__main__":
    main()
