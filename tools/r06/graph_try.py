"""Can one join step (build_table + probe_relation on a reserved context) be
captured into a HIP graph and replayed?  For each size: eager step time vs
graph replay time (both back to back, no host sync inside), and the replayed
result vs the oracle.  Prints one line per (size, strategy)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mlir-hashjoin_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hashjoin  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def one(n, strategy, reps=50):
    rk, rp, sk, sp = O.gen_pkfk_i64(77, n, n, 1.0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    rk, rp, sk, sp = d(rk), d(rp), d(sk), d(sp)
    hj = hashjoin.HashJoin(0)
    hj.set_strategy(strategy)
    hj.allocate_hash_table(n, 64)
    hj.build_table(rk, rp)
    hj.reserve_probe(n, 64)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(reps):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / reps * 1e3
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    except Exception as e:  # noqa: BLE001
        print(f"n=2^{n.bit_length() - 1} {strategy}: capture failed: {type(e).__name__}: {str(e)[:300]}", flush=True)
        torch.cuda.synchronize()
        hj.close()
        return
    out_r.fill_(-1)
    cnt.zero_()
    g.replay()
    torch.cuda.synchronize()
    m = int(cnt.item())
    # PK-FK at f = 1, payload = row index on both sides: every S row once,
    # each with the R row holding its key
    o_r, o_s = out_r[:m].cpu().numpy(), out_s[:m].cpu().numpy()
    hk_r, hk_s = rk.cpu().numpy(), sk.cpu().numpy()
    ok = m == n and (np.sort(o_s) == np.arange(n)).all() and (hk_r[o_r] == hk_s[o_s]).all()
    if ok and n <= 1 << 16:
        er, es = O.chained_join_i64(rk.cpu().numpy(), rp.cpu().numpy(), sk.cpu().numpy(), sp.cpu().numpy(), H=n)
        ok = O.same_multiset(o_r, o_s, er, es)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / reps * 1e3
    print(f"n=2^{n.bit_length() - 1} {strategy} used={hj.strategy_used}: eager {eager:.4f} ms/step, graph replay "
          f"{graph:.4f} ms/step, replay parity {'ok' if ok else 'FAILED'} (M={m})", flush=True)
    del g
    hj.close()


if __name__ == "__main__":
    for lg in (12, 16, 20, 22):
        for strat in ("auto", "radix", "global"):
            one(1 << lg, strat)
