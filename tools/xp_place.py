"""Placement probe A/B: C3 build + probe on ten fresh contexts in one process
(each context allocates new bucket sets), phase times per context and the
probe's counts.  Run once with HJ_PLACEMENT_PROBE=0 and once without.
    python tools/xp_place.py [contexts] [config] > out.jsonl
"""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "mlir-hashjoin_amd"))
import bench  # noqa: E402
import hashjoin  # noqa: E402


def run(rk, rp, sk, sp, wide, cap, steps=5):
    hj = hashjoin.HashJoin(0)
    hj.allocate_hash_table(rk.numel(), 64 if wide else 32)
    hj.reserve_probe(sk.numel(), 64 if wide else 32)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    out_r = torch.empty(max(cap, 1), dtype=torch.int64 if wide else torch.int32, device="cuda")
    out_s = torch.empty_like(out_r)
    hj.set_timing(True)
    acc = {}
    for i in range(2 + steps):
        hj.build_table(rk, rp)
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
        t = hj.last_timing()
        if i >= 2:
            for k in ("build", "probe_partition", "probe_join"):
                acc[k] = acc.get(k, 0.0) + t[k] / steps
    assert int(cnt.item()) <= cap
    hj.close()
    del out_r, out_s
    torch.cuda.empty_cache()
    return {k: round(v, 4) for k, v in acc.items()}


def main():
    nctx = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C3"
    NR, NS, distn, ktype, _ = bench.CONFIGS[cfg]
    wide = ktype == "int64"

    class A:
        seed = 42
    rk, rp, sk, sp = bench.gen_inputs(hashjoin, A, NR, NS, distn, 0, NR, 0, NS)
    torch.cuda.synchronize()
    # output capacity: |S| for the key joins, else the exact M of one count
    cap = bench.expected_rows(distn, NR, NS)
    if cap is None:
        hj = hashjoin.HashJoin(0)
        hj.allocate_hash_table(NR, 64 if wide else 32)
        hj.build_table(rk, rp)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        hj.probe_relation(sk, sp, None, None, count=cnt)
        cap = int(cnt.item())
        hj.close()
    for k in range(nctx):
        r = run(rk, rp, sk, sp, wide, cap)
        r["ctx"] = k
        r["config"] = cfg
        r["placement"] = hashjoin.placement_stats()
        r["probe_env"] = os.environ.get("HJ_PLACEMENT_PROBE", "1")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
