"""Owner-routing (hj.partition) throughput on one MI355X: |rows| x parts
cases, inputs resident in HBM, median of 10 timed calls after 2 warm-ups
(wall clock around a device sync).  Bytes = key + payload read (hist reads
the key column again) + 16-B tuples written.  profiles/r02_route_tiles.txt
holds the tile-shape comparison it was written for.

usage: python tools/route_ab.py
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402


def main():
    hj = hashjoin.HashJoin(0)
    for lg in (25, 28):
        n = 1 << lg
        g = torch.Generator(device="cuda").manual_seed(7)
        key = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device="cuda", generator=g)
        pay = torch.arange(n, dtype=torch.int64, device="cuda")
        out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        for P in (1, 2, 4, 8, 64, 128):
            counts = torch.empty(P, dtype=torch.int64, device="cuda")
            ts = []
            for it in range(12):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hj.partition(key, pay, P, out=out, counts=counts)
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(time.perf_counter() - t0)
            ms = statistics.median(ts) * 1e3
            assert int(counts.sum()) == n
            print(json.dumps({"rows": f"2^{lg}", "parts": P, "ms": round(ms, 4), "GBps": round(n * 40 / ms / 1e6, 1)}), flush=True)
        del key, pay, out


if __name__ == "__main__":
    main()
