"""Diagnostic: RCCL (torch nccl backend) collectives used by hashjoin.dist on
this box, one step at a time with timestamps (world size from torchrun)."""
import os, sys, time
import torch, torch.distributed as dist
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}s rank{os.environ.get('RANK','0')}]", *a, file=sys.stderr, flush=True)
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
use_dev = os.environ.get("DEVICE_ID", "1") == "1"
log("init_process_group device_id" if use_dev else "init_process_group (lazy)")
if use_dev:
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
else:
    dist.init_process_group("nccl")
w = dist.get_world_size()
log("world", w)
x = torch.arange(2 * w, dtype=torch.int64, device="cuda")
y = torch.empty_like(x)
dist.all_to_all_single(y, x); torch.cuda.synchronize(); log("a2a equal splits ok", y.tolist())
z = torch.empty(3 * w, dtype=torch.int64, device="cuda")
dist.all_to_all_single(z, torch.arange(3 * w, dtype=torch.int64, device="cuda"), [3] * w, [3] * w)
torch.cuda.synchronize(); log("a2a split sizes ok")
t = torch.ones(1, device="cuda"); dist.all_reduce(t); torch.cuda.synchronize(); log("all_reduce ok", t.item())
dist.barrier(); log("barrier ok")
dist.destroy_process_group(); log("done")
