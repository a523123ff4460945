"""Join time on sequential int64 keys (R = 0..n-1 in order, S = a random
sample of them): a common primary-key shape, and one where a multiplicative
hash's bits are far from random.  Prints the radix join's per-call time
(median of 5 after 1 warm-up, wall clock around a sync).

usage: HJ_JOIN_BKT=0|1 python tools/seqkeys_ab.py [log2 rows]
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlir-hashjoin_amd"))
import torch  # noqa: E402

import hashjoin  # noqa: E402


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    n = 1 << lg
    hj = hashjoin.HashJoin(0)
    rk = torch.arange(n, dtype=torch.int64, device="cuda")
    rp = rk.clone()
    g = torch.Generator(device="cuda").manual_seed(3)
    sk = torch.randint(0, n, (n,), dtype=torch.int64, device="cuda", generator=g)
    sp = torch.arange(n, dtype=torch.int64, device="cuda")
    ts = []
    for it in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o_r, o_s = hj.join(rk, rp, sk, sp)
        torch.cuda.synchronize()
        if it:
            ts.append(time.perf_counter() - t0)
    assert o_r.numel() == n and bool((rk[o_r] == sk[o_s]).all())
    print(f"HJ_JOIN_BKT={os.environ.get('HJ_JOIN_BKT', '1')} 2^{lg} sequential keys: {statistics.median(ts) * 1e3:.3f} ms, "
          f"duplicates={hj.has_duplicates()}")


if __name__ == "__main__":
    main()
