"""Diagnostic: can two ranks share one GPU under RCCL on this box?  (If so,
the multi-rank exchange of hashjoin.dist can run on a one-GPU box.)  Every
rank uses device LOCAL_RANK % device_count."""
import os, sys, time
import torch, torch.distributed as dist
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}s rank{os.environ.get('RANK','0')}]", *a, file=sys.stderr, flush=True)
local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
w, r = dist.get_world_size(), dist.get_rank()
log("world", w, "device", local)
x = torch.arange(2 * w, dtype=torch.int64, device="cuda") + 100 * r
y = torch.empty_like(x)
dist.all_to_all_single(y, x); torch.cuda.synchronize(); log("a2a ok", y.tolist())
src = torch.full((1000,), r, dtype=torch.int64, device="cuda")
dst = torch.empty(1000, dtype=torch.int64, device="cuda")
ops = [dist.P2POp(dist.isend, src, (r + 1) % w), dist.P2POp(dist.irecv, dst, (r - 1) % w)]
for q in dist.batch_isend_irecv(ops): q.wait()
torch.cuda.synchronize(); log("p2p ok", dst[0].item())
dist.barrier(); log("barrier ok")
dist.destroy_process_group(); log("done")
