#!/usr/bin/env python3
"""bench.py -- hash-join throughput on MI355X (BASELINE.json metric).

Metric: probed tuples/s (+ joined rows/s), |R| = |S| = 2^28 int64 key +
int64 payload, PK-FK synthetic relations (SURVEY 8(d) C3 shape: R keys
unique, every S row matches exactly one R row).  One step = one complete
join of the whole relations with inputs resident in HBM:

  N = 1 : table init + build + probe (one GPU holds everything: ~22 GiB)
  N > 1 : radix partition R and S -> RCCL all-to-all of 16-B tuples ->
          local init + build + probe (strong scaling: the GLOBAL relations
          stay 2^28 x 2^28; each rank generates its 1/N slice)

value = |S| / (time per step), the whole job over all ranks (max over ranks).
Launch:  python bench.py [--gpus 1 --steps K --warmup W]
         python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (log2 |R|, log2 |S|, distribution, description)
    "C3": (28, 28, "pkfk", "PK-FK |R|=|S|=2^28 int64 key+payload, match fraction 1"),
    "C1": (26, 26, "pkfk", "PK-FK |R|=|S|=2^26 int64 key+payload, match fraction 1"),
    "C1-ref": (26, 26, "uniform", "uniform keys in [1,2^30] both sides, |R|=|S|=2^26 int64"),
    "C2": (20, 30, "pkfk", "PK-FK |R|=2^20 build, |S|=2^30 probe, int64"),
    "C4": (28, 28, "zipf", "PK build |R|=2^28, Zipf(0.9) foreign keys |S|=2^28, int64"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log2", type=int, default=22)
    ap.add_argument("--verify", action="store_true", help="check the last step's output properties")
    ap.add_argument("--strategy", default="auto", choices=["auto", "global", "radix"])
    ap.add_argument("--radix-bits", type=int, default=0)
    ap.add_argument("--force-dist", action="store_true",
                    help="use the multi-GPU code path (partition + all-to-all) even at N=1")
    return ap.parse_args()


def cpu_baseline(seed, log2n, threads):
    """The reference's join_v2 (chained table, key urem H with H = |R|/100 as
    join-performances.md:3,8, count -> block scan -> staged probe) restated on
    host threads (oracle/, test infrastructure), timed on a bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import pyoracle as O
    n = 1 << log2n
    rk, rp, sk, sp = O.gen_pkfk_i64(seed, n, n)
    H = max(1, n // 100)
    O.chained_join_i64_omp(rk[:4096], rp[:4096], sk[:4096], sp[:4096], 41, threads)   # warm the pool
    t0 = time.perf_counter()
    m, ph = O.chained_join_i64_omp(rk, rp, sk, sp, H, threads)
    dt = time.perf_counter() - t0
    assert m == n, (m, n)
    return {"value": n / dt, "unit": "probe tuples/s", "cores": threads, "kind": "port",
            "sample": f"|R|=|S|=2^{log2n} PK-FK int64, H=|R|/100 (reference ratio), join_v2 restated "
                      f"(oracle/hj_oracle.c) on {threads} host threads; {dt:.2f} s "
                      f"(init {ph[0]:.2f} / build {ph[1]:.2f} / count {ph[2]:.2f} / probe {ph[3]:.2f} s)"}


def pmc_traffic(config, n_gpus, kernel):
    """HBM bytes per launch of `kernel` for this workload from the committed
    rocprofv3 PMC summary (profiles/pmc_latest.json, written by
    profiles/pmc_to_json.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(f"{config}/n{n_gpus}", {}).get("kernels", {}).get(kernel)
        return None if e is None else e.get("hbm_bytes_per_launch")
    except (OSError, ValueError, AttributeError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    use_dist = world > 1 or a.force_dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)

    import hashjoin
    from hashjoin.dist import distributed_join

    lr, ls, distn, desc = CONFIGS[a.config]
    NR, NS = 1 << lr, 1 << ls
    r0, nr = rank * NR // world, (rank + 1) * NR // world - rank * NR // world
    s0, ns = rank * NS // world, (rank + 1) * NS // world - rank * NS // world
    if distn == "pkfk":
        rk, rp, sk, sp = hashjoin.gen_pkfk(a.seed, NR, NS, 1.0, r0, nr, s0, ns)
    elif distn == "zipf":
        rk, rp, _, _ = hashjoin.gen_pkfk(a.seed, NR, NS, 1.0, r0, nr, s0, 0)
        sk, sp = hashjoin.gen_zipf(a.seed, NR, NS, 0.9, s0, ns)
    else:
        rk, rp = hashjoin.gen_uniform_i64(a.seed, 1, 1, 1 << 30, nr, i0=r0)
        sk, sp = hashjoin.gen_uniform_i64(a.seed, 2, 1, 1 << 30, ns, i0=s0)
    hj = hashjoin.HashJoin(local)
    hj.set_strategy(a.strategy, radix_bits=a.radix_bits)
    expect_m = NS if distn in ("pkfk", "zipf") else None
    torch.cuda.synchronize()

    phases = {"init": 0.0, "build": 0.0, "probe": 0.0, "probe_partition": 0.0, "probe_join": 0.0, "route": 0.0,
              "partition+exchange": 0.0}
    last = {}

    if not use_dist:
        hj.allocate_hash_table(NR, 64)
        hj.build_table(rk, rp)
        hj.reserve_probe(NS, 64)
        cap = NS if distn in ("pkfk", "zipf") else int(NR * NS / (1 << 30) * 1.1) + 4096
        out_r = torch.empty(cap, dtype=torch.int64, device="cuda")
        out_s = torch.empty_like(out_r)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        hj.set_timing(True)

        def step(acc):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
            t = hj.last_timing()          # synchronises: the step ends with M known on the host
            if acc:
                for k in ("init", "build", "probe", "probe_partition", "probe_join"):
                    phases[k] += max(0.0, t[k])
            last["m"] = int(cnt.item())
    else:
        # strong scaling over the GLOBAL relations; output stays distributed
        hj.allocate_hash_table(2 * nr, 64)

        def step(acc):
            ev = {}
            o_r, o_s = distributed_join(hj, rk, rp, sk, sp, phases=ev)
            ev["probed"].synchronize()
            if acc:
                # transfers overlap compute (hashjoin.dist): R's tuples move
                # during S's routing, S's during R's build
                phases["route"] += ev["start"].elapsed_time(ev["routed"])
                phases["build"] += ev["routed"].elapsed_time(ev["built"])
                phases["probe"] += ev["built"].elapsed_time(ev["probed"])
            last["m"] = o_r.numel()
            last["rows"] = ev["rows"]
            last["out"] = (o_r, o_s)

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    m_local = last["m"]
    if use_dist:
        tt = torch.tensor([elapsed, float(m_local)], dtype=torch.float64, device="cuda")
        mx = tt.clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item()); m_total = int(sm[1].item())
    else:
        m_total = m_local
    if expect_m is not None and m_total != expect_m:
        raise SystemExit(f"join produced {m_total} rows, expected {expect_m}")

    if a.verify and not use_dist:
        o_r, o_s = out_r[:m_local], out_s[:m_local]
        assert bool((rk[o_r] == sk[o_s]).all()), "non-matching pair in output"

    ms = elapsed * 1000.0 / a.steps
    value = NS / (ms / 1000.0)
    ph = {k: round(v / a.steps, 4) for k, v in phases.items() if v > 0}

    # Roofline of the dominant kernel (DESIGN.md "Measurement").  Radix: k_join,
    # the longest single launch; algorithmic bytes per launch = 16 B per R row
    # + 16 B per S row read once + 16 B per output pair (= 48 B per probe row
    # at |R| = |S|, f = 1).  Global table: k_probe, 16 B S row + 16 B slot +
    # 16 B output per probe row.  Duration: HIP events on the
    # launch stream around the join (probe_join phase).
    probe_ms = phases["probe"] / a.steps
    join_ms = phases["probe_join"] / a.steps
    build_ms = (phases["init"] + phases["build"]) / a.steps
    strategy = hj.strategy_used or a.strategy
    if use_dist:
        # per-kernel events are not recorded through the distributed path:
        # the probe phase (S partition + k_join on the received tuples)
        nr_loc, ns_loc = last["rows"]
        kern, join_ms = "probe phase (local S partition + k_join)", probe_ms
        kbytes = (nr_loc + ns_loc) * 16 + m_local * 16
    elif strategy == "radix":
        kern, kbytes = "k_join", (nr + ns) * 16 + m_local * 16
    else:
        kern, kbytes = "k_probe", ns * 32 + m_local * 16
    achieved = kbytes / (join_ms / 1000.0) / 1e9 if join_ms > 0 else None
    probe_bytes = ns * 32 + m_local * 16   # 48 B per probe row at f = 1
    passes = hj.radix_passes if strategy == "radix" else 0
    line = {
        "metric": "probed tuples/sec + joined rows/sec, |R|=|S|=2^28 int64 keys",
        "value": round(value, 1),
        "unit": "probe tuples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (counter-based PK-FK generator, seed 0x5EED, generated on device)",
        "config": {"workload": f"{a.config}: {desc}", "R_rows": NR, "S_rows": NS, "key": "int64",
                   "payload": "int64", "distribution": distn,
                   "parallelism": ("single GPU" if not use_dist
                                   else f"radix-partitioned x{world}, RCCL all-to-all")},
        "joined_rows_per_sec": round(m_total / (ms / 1000.0), 1),
        "result_rows": m_total,
        "phase_ms": ph,
        "strategy": strategy,
        "roofline": {
            "kernel": kern if use_dist else f"{kern} ({'hj_radix.hip' if kern == 'k_join' else 'hj_kernels.hip'})",
            "bound": "hbm",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": pmc_traffic(a.config, world, kern),
            "algorithmic_bytes_per_launch": kbytes,
            "avg_launch_ms": round(join_ms, 4),
        },
        # the whole probe phase (S partition passes + join for radix) at
        # SURVEY 8(d)'s 48 B per probe row
        "probe_phase": {
            "achieved": round(probe_bytes / (probe_ms / 1000.0) / 1e9, 1) if probe_ms > 0 else None,
            "frac": round(probe_bytes / (probe_ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 4) if probe_ms > 0 else None,
            "unit": "GB/s", "algorithmic_bytes": probe_bytes, "ms": round(probe_ms, 4),
        },
        # build phase: radix = R partition passes, each reading and writing 16 B per row
        "build_phase": {
            "kernel": f"k_pass x{passes}" if strategy == "radix" else "k_init + k_build",
            "algorithmic_bytes": nr * 32 * max(1, passes),
            "achieved": round(nr * 32 * max(1, passes) / (build_ms / 1000.0) / 1e9, 1) if build_ms > 0 else None,
            "unit": "GB/s", "ms": round(build_ms, 4),
        },
    }
    if rank == 0 and not use_dist and not a.no_cpu_baseline:
        threads = min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        line["cpu_baseline"] = cpu_baseline(a.seed, a.cpu_sample_log2, threads)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    hj.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
