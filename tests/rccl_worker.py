"""Single-rank RCCL worker for tests/test_gpu_dist.py (run as its own
process: the process group is created before anything touches the GPU).

  distributed_join over a world-size-1 "nccl" (= RCCL) group vs the oracle:
  shuffle mode with the rank's own slice sent through RCCL point-to-point
  (self send/recv, cut into pieces), replicate mode, repeated build keys,
  INT64_MIN keys, an undersized output; then one >1 GiB self-exchange at the
  default piece size, compared byte for byte (the 4 GiB-message truncation
  fixed in e8c2a74)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "mlir-hashjoin_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29641")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import numpy as np
    import hashjoin
    from hashjoin.dist import Exchange, MAX_ROWS_PER_ROUND, distributed_join
    from oracle import pyoracle as O

    hj = hashjoin.HashJoin(0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    I64_MIN = -(1 << 63)
    cases = {
        "pkfk": lambda: O.gen_pkfk_i64(41, 30000, 50000, 0.8),
        "dups": lambda: O.gen_uniform_i64(42, 1, 1, 700, 20000) + O.gen_uniform_i64(42, 2, 1, 700, 15000),
        "int64_min": lambda: O.gen_uniform_i64(43, 1, I64_MIN, I64_MIN + 300, 9000)
        + O.gen_uniform_i64(43, 2, I64_MIN, I64_MIN + 300, 7000),
    }
    ok = 0
    for name, gen in cases.items():
        rk, rp, sk, sp = gen()
        er, es = O.nested_loop_i64(rk, rp, sk, sp)
        for mode, kw in (("shuffle", dict(replicate_max_rows=0, max_rows=4093, self_p2p=True)),
                         ("shuffle_copy", dict(replicate_max_rows=0)),
                         ("replicate", dict(replicate_max_rows=1 << 21)),
                         ("resize", dict(replicate_max_rows=0, capacity=3, self_p2p=True)),
                         ("s_parts", dict(replicate_max_rows=0, max_rows=2999, self_p2p=True, s_parts=3)),
                         ("s_parts_overflow", dict(replicate_max_rows=0, self_p2p=True, s_parts=2, capacity=2000)),
                         # the folded routing (rows arrive first-pass partitioned)
                         ("folded", dict(replicate_max_rows=0, route_bits=4, max_rows=3001, self_p2p=True)),
                         ("folded_parts", dict(replicate_max_rows=0, route_bits=5, self_p2p=True, s_parts=3)),
                         ("folded_alias", dict(replicate_max_rows=0, route_bits=3, s_parts=2, capacity=1500))):
            ph = {}
            o_r, o_s = distributed_join(hj, d(rk), d(rp), d(sk), d(sp), phases=ph, **kw)
            torch.cuda.synchronize()
            got_r, got_s = o_r.cpu().numpy(), o_s.cpu().numpy()
            assert O.same_multiset(got_r, got_s, er, es), (name, mode, len(got_r), len(er))
            assert ph["mode"] == ("replicate" if mode == "replicate" else "shuffle")
            assert ph.get("folded", False) == mode.startswith("folded")
            ok += 1
            print(f"ok {name} {mode} M={len(er)}", flush=True)
    # >1 GiB self-exchange at the default piece size: two RCCL messages
    n = MAX_ROWS_PER_ROUND + 12345
    send = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    send[:, 0] = torch.arange(n, device="cuda")
    send[:, 1] = send[:, 0] * 0x9E3779B1 + 7
    x = Exchange(send, torch.tensor([n], dtype=torch.int64, device="cuda"), self_p2p=True)
    recv = x.wait()
    torch.cuda.synchronize()
    assert recv.shape == send.shape and torch.equal(recv, send), "self-exchange corrupted"
    print(f"ok self-exchange {n} rows = {n * 16 / 2**30:.3f} GiB in 2 pieces", flush=True)
    hj.close()
    dist.destroy_process_group()
    print(f"RCCL_WORKER_OK {ok + 1}", flush=True)


if __name__ == "__main__":
    main()
