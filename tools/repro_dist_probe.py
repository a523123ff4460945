"""Diagnostic: the distributed path's local steps without RCCL, timed one by one."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlir-hashjoin_amd"))
import torch
import hashjoin
t0 = time.time()
def log(*a):
    torch.cuda.synchronize()
    print(f"[{time.time()-t0:7.2f}s]", *a, file=sys.stderr, flush=True)
lg = int(os.environ.get("LG", "28")); n = 1 << lg
mode = os.environ.get("MODE", "tuples")
if os.environ.get("RCCL", "0") != "0":
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
    x = torch.ones(4, device="cuda"); dist.all_reduce(x); log("rccl up", x.tolist())
rk, rp, sk, sp = hashjoin.gen_pkfk(0x5EED, n, n)
hj = hashjoin.HashJoin(0)
if os.environ.get("RESERVE", "1") == "1":
    hj.allocate_hash_table(2 * n, 64)
log("gen", mode)
if mode == "exchange":
    from hashjoin.dist import exchange
    tr, cr = hj.partition(rk, rp, 1); ts, cs = hj.partition(sk, sp, 1)
    rr, rs, _ = exchange(tr, cr, ts, cs); log("exchanged", bool(torch.equal(rr, tr)), bool(torch.equal(rs, ts)))
    hj.build_tuples(rr); log("built", hj.strategy_used)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    m = int(hj.probe_tuples(rs, out_r, out_s).item()); log("probed", m)
elif mode == "routed":
    tr, cr = hj.partition(rk, rp, 1); ts, cs = hj.partition(sk, sp, 1)
    log("routed", cr.tolist(), cs.tolist())
    hj.build_tuples(tr); log("built", hj.strategy_used)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    m = int(hj.probe_tuples(ts, out_r, out_s).item()); log("probed", m)
elif mode == "tuples":
    tr = torch.stack([rk, rp], 1).contiguous(); ts = torch.stack([sk, sp], 1).contiguous()
    log("packed")
    hj.build_tuples(tr); log("built", hj.strategy_used)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    m = int(hj.probe_tuples(ts, out_r, out_s).item()); log("probed", m)
else:
    hj.build_table(rk, rp); log("built", hj.strategy_used)
    out_r = torch.empty(n, dtype=torch.int64, device="cuda"); out_s = torch.empty_like(out_r)
    m = int(hj.probe_relation(sk, sp, out_r, out_s).item()); log("probed", m)
