#!/usr/bin/env python3
"""bench.py -- hash-join throughput on MI355X (BASELINE.json metric).

Metric: probed tuples/s (+ joined rows/s), |R| = |S| = 2^28 int64 key +
int64 payload, PK-FK synthetic relations (SURVEY 8(d) C3 shape: R keys
unique, every S row matches exactly one R row).  One step = one complete
join of the whole relations with inputs resident in HBM:

  N = 1 : build (R radix partition) + probe (S radix partition + LDS join)
  N > 1 : radix-route R and S -> RCCL all-to-all of 16-B tuples -> local
          build + probe (strong scaling: the GLOBAL relations stay
          2^28 x 2^28; each rank generates its 1/N slice).  Build sides of
          <= 2^21 rows are all-gathered instead (no S shuffle).

value = |S| / (time per step), the whole job over all ranks (max over ranks).
`roofline` is SURVEY 8(d)'s probe-phase figure: 48 B per probe tuple (16 B S
row + 16 B slot + 16 B output pair) over the probe phase's HIP-event time;
`roofline.read_frac` counts the probe phase's READ bytes only (16 B S row +
16 B slot per probe tuple: north_star's "HBM read roofline").
`roofline.kernel` is the same for the dominant kernel (the LDS join: the one
hj_ctx_join_kernel names -- k_join_b / k_join_u / k_join_grp) alone.
Launch:  python bench.py [--gpus 1 --steps K --warmup W --config C3]
         python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mlir-hashjoin_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
HBM_ACHIEVABLE_GBS = 6290.0   # same guide: float4 copy, measured

CONFIGS = {
    # name: (|R|, |S|, distribution, key type, description)
    "C3": (1 << 28, 1 << 28, "pkfk", "int64", "PK-FK |R|=|S|=2^28 int64 key+payload, match fraction 1"),
    "C1": (1 << 26, 1 << 26, "pkfk", "int64", "PK-FK |R|=|S|=2^26 int64 key+payload, match fraction 1"),
    "C1-ref": (1 << 26, 1 << 26, "uniform30", "int64", "uniform keys in [1,2^30] both sides, |R|=|S|=2^26 int64"),
    "C2": (1 << 20, 1 << 30, "pkfk", "int64", "PK-FK |R|=2^20 build, |S|=2^30 probe, int64"),
    "C4": (1 << 28, 1 << 28, "zipf", "int64", "PK build |R|=2^28, Zipf(0.9) foreign keys |S|=2^28, int64"),
    # the reference's own published workloads (join-performances.md:3-6 / :16-19 and :8-11 / :21-24),
    # in its types: i32 keys, row-id payloads, (rowR, rowS) i32 output
    "REF-A": (10_000_000, 10_000_000, "ref100k", "int32",
              "reference workload 1: 10M x 10M i32 keys uniform in [1, 100k] (~1e9 result rows)"),
    "REF-B": (100_000_000, 100_000_000, "ref1e9", "int32",
              "reference workload 2: 100M x 100M i32 keys uniform in [1, 1e9] (~1e7 result rows)"),
    # workload 1's key distribution as int64 key + payload columns: most build
    # keys repeat (~100 copies), the int64 rows' mostly-repeated join path
    "REF-A64": (10_000_000, 10_000_000, "ref100k64", "int64",
                "workload 1's keys as int64 key+payload: 10M x 10M keys uniform in [1, 100k] (~1e9 result rows)"),
}
# the reference's own times for those workloads (join-performances.md; sm_86, all four kernels + module loads)
REFERENCE_PUBLISHED = {
    "REF-A": {"join_v1_s": 2.0, "join_v2_s": 1.5, "source": "join-performances.md:3-6, :16-19"},
    "REF-B": {"join_v1_s": 12.0, "join_v2_s": 12.5, "source": "join-performances.md:8-11, :21-24"},
}
# probe phase: S partition passes + the LDS join (hj_ctx_join_kernel: k_join_b /
# k_join_u / k_join_grp; k_join takes the items they defer -- none at C1-C4 --
# and is counted when it ran; the kernels not chosen exit at once)
PROBE_KERNELS = ("k_pass",)
FAST_JOIN_KERNELS = ("k_join_b", "k_join_u", "k_join_grp")
OPTIONAL_PROBE_KERNELS = FAST_JOIN_KERNELS + ("k_join",)

# roofline scopes.  t_probe always contains EVERY partition
# pass of S: on the distributed path S's first pass runs inside its routing
# (the EXACT k_pass), so the t_probe figure there adds S's route time; the
# local-only figure is reported beside it under its own name.
SCOPE_T_PROBE = "probe phase: S radix partition passes + the LDS join (SURVEY 8(d) t_probe)"
SCOPE_T_PROBE_DIST = ("probe phase incl. S's routing (SURVEY 8(d) t_probe, every S partition pass): S's route "
                      "(k_slot_hist + EXACT k_pass + count exchange) + S's local k_pass + the LDS join")
SCOPE_LOCAL_PROBE = ("local probe only, NOT t_probe: S's local (second) k_pass + the LDS join; S's first "
                     "partition pass ran in the route phase")
SCOPE_GLOBAL = "probe phase: k_probe + k_probe_slow (global table)"
COPY_FLOOR_ROWS = 1 << 28   # 16-B rows: 4 GiB read + 4 GiB written = one C3 partition pass's bytes


def frac_of(b, t_ms, peak=HBM_PEAK_GBS):
    return round(b / (t_ms / 1000.0) / 1e9 / peak, 4) if t_ms and t_ms > 0 else None


def probe_roofline(strategy, use_dist, probe_ms, s_route_ms, probe_bytes, read_bytes, structure_bytes=None,
                   floor=None):
    """The probe-phase roofline record.  probe_ms: the probe
    phase's HIP-event time; s_route_ms: S's routing on the distributed path
    (0 otherwise); structure_bytes: the phase's structural HBM bytes (every
    S pass + the join), priced at the box's own copy rates from `floor`."""
    dist_t = bool(use_dist and s_route_ms)
    t = probe_ms + (s_route_ms if dist_t else 0.0)
    if strategy != "radix":
        scope = SCOPE_GLOBAL
    else:
        scope = SCOPE_T_PROBE_DIST if dist_t else SCOPE_T_PROBE
    roof = {
        "scope": scope,
        "bound": "hbm",
        "achieved": round(probe_bytes / (t / 1000.0) / 1e9, 1) if t > 0 else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": frac_of(probe_bytes, t),
        "algorithmic_bytes": probe_bytes,
        "ms": round(t, 4),
        "frac_of_achievable": frac_of(probe_bytes, t, HBM_ACHIEVABLE_GBS),
        # north_star's "HBM read roofline": the probe phase's algorithmic READ
        # bytes only (S row + one slot per probe tuple)
        "read_bytes": read_bytes,
        "read_frac": frac_of(read_bytes, t),
        "target": "north_star: frac >= 0.40 at |R|=|S|=2^28 (t_probe <= 4.0 ms)",
    }
    if dist_t:
        roof["s_route_ms"] = round(s_route_ms, 4)
        roof["local_probe"] = {"scope": SCOPE_LOCAL_PROBE, "ms": round(probe_ms, 4),
                               "frac": frac_of(probe_bytes, probe_ms)}
    if floor and structure_bytes and strategy == "radix":
        fl = structure_bytes / (floor["persistent_gbs"] * 1e6)
        ff = structure_bytes / (floor["flat_gbs"] * 1e6)
        roof["structure_bytes"] = int(structure_bytes)
        roof["floor_ms"] = round(fl, 4)
        roof["floor_flat_ms"] = round(ff, 4)
        roof["phase_over_floor"] = round(t / fl, 4) if fl > 0 else None
        roof["phase_over_flat_floor"] = round(t / ff, 4) if ff > 0 else None
        roof["floor_note"] = ("structure_bytes (every S pass + the join's R, S and pairs) at this box's own "
                              "copy rates, measured in-process before the warm-up (copy_floor)")
    return roof


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log2", type=int, default=22)
    ap.add_argument("--no-host-leg", action="store_true", help="skip the host-memref (PCIe-inclusive) leg")
    ap.add_argument("--verify", action="store_true", help="check the last step's output properties")
    ap.add_argument("--strategy", default="auto", choices=["auto", "global", "radix"])
    ap.add_argument("--radix-bits", type=int, default=0)
    ap.add_argument("--force-dist", action="store_true",
                    help="use the multi-GPU code path (partition + all-to-all) even at N=1")
    ap.add_argument("--s-parts", type=int, default=0,
                    help="multi-GPU path: batches the shuffled probe side moves in (0: hashjoin.dist default)")
    ap.add_argument("--no-floor", action="store_true", help="skip the in-process copy floor (roofline.floor_ms)")
    ap.add_argument("--log2", type=int, default=0,
                    help="experiments: |R| = |S| = 2^LOG2 rows instead of the config's sizes (not a bench line)")
    return ap.parse_args()


# ---------------------------------------------------------------- CPU baseline
def host_facts():
    """Cores this process may use on the host (affinity and cgroup quota) and
    the CPU model, as SURVEY 8(d) asks the CPU baseline to state."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = platform.processor() or ""
    try:
        for line in subprocess.check_output(["lscpu"], text=True, timeout=10).splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": aff, "cpu_count": os.cpu_count(), "cgroup_cpus": quota, "usable_cores": usable,
            "lscpu_model": model}


def cpu_baseline(seed, log2n):
    """The reference's algorithms restated on the host (oracle/hj_oracle.c,
    test infrastructure), each timed on a bounded sample:
      * join_v2 (join_v2.mlir:227-604: chained table, key urem H, count ->
        block scan -> staged probe) at H = |R|/100 (the reference's ratio,
        join-performances.md:3,8) and H = |R|, on all usable cores and on 1;
      * the nested loop (shared.cpp:154-165, nested-loop.mlir:29-192) up to
        2^16 x 2^16, extrapolated quadratically to 2^28 x 2^28 (labelled);
      * the reference's own compiled check() (its nested loop + sort, kind
        "reference") at 2^16 x 2^16 i32 on 1 core, when oracle/_ref is built."""
    sys.path.insert(0, ROOT)
    from oracle import pyoracle as O
    facts = host_facts()
    allc = facts["usable_cores"]
    runs = []

    def v2(log2, H_div, threads):
        n = 1 << log2
        rk, rp, sk, sp = O.gen_pkfk_i64(seed, n, n)
        H = max(1, n // H_div)
        O.chained_join_i64_omp(rk[:4096], rp[:4096], sk[:4096], sp[:4096], 41, threads)   # warm the pool
        t0 = time.perf_counter()
        m, ph = O.chained_join_i64_omp(rk, rp, sk, sp, H, threads)
        dt = time.perf_counter() - t0
        assert m == n, (m, n)
        probe_s = ph[2] + ph[3]
        runs.append({"algorithm": "join_v2 restated", "H": f"|R|/{H_div}" if H_div > 1 else "|R|",
                     "rows": f"2^{log2} x 2^{log2}", "threads": threads, "seconds": round(dt, 3),
                     "probe_tuples_per_s": round(n / probe_s, 1) if probe_s > 0 else None,
                     "joined_rows_per_s": round(m / dt, 1),
                     "phases_s": {"init": round(ph[0], 4), "build": round(ph[1], 4), "count": round(ph[2], 4),
                                  "probe": round(ph[3], 4)}})
        return runs[-1]

    def nested(log2, threads):
        n = 1 << log2
        rk, _, sk, _ = O.gen_pkfk_i64(seed, n, n)
        L = O.lib()
        t0 = time.perf_counter()
        m = L.oracle_nested_loop_count_i64_omp(rk.ctypes.data, n, sk.ctypes.data, n, threads)
        dt = time.perf_counter() - t0
        assert m == n, (m, n)
        ext = dt * (2.0 ** (28 - log2)) ** 2
        runs.append({"algorithm": "nested loop restated", "rows": f"2^{log2} x 2^{log2}", "threads": threads,
                     "seconds": round(dt, 3), "probe_tuples_per_s": round(n / dt, 1),
                     "extrapolated_2p28": {"seconds": round(ext, 1), "probe_tuples_per_s": round((1 << 28) / ext, 2),
                                           "note": "quadratic extrapolation from the measured sample, not measured"}})
        return runs[-1]

    def ref_nested(log2):
        # the reference's OWN compiled CPU join: check() (shared.cpp:129-172,
        # built from its sources into oracle/_ref/shared.so) runs the nested
        # loop over i32 keys and compares its sorted pairs with ours
        import numpy as np
        n = 1 << log2
        rng = np.random.default_rng(seed)
        r = rng.permutation(n).astype(np.int32) + 1
        ps = rng.permutation(n)
        s = r[ps]
        t0 = time.perf_counter()
        ok = O.ref_check(r, s, ps.astype(np.int32), np.arange(n, dtype=np.int32))
        dt = time.perf_counter() - t0
        assert ok == 1, ok
        ext = dt * (2.0 ** (28 - log2)) ** 2
        runs.append({"algorithm": "reference check() nested loop (oracle/_ref/shared.so)", "kind": "reference",
                     "rows": f"2^{log2} x 2^{log2} i32", "threads": 1, "seconds": round(dt, 3),
                     "probe_tuples_per_s": round(n / dt, 1),
                     "extrapolated_2p28": {"seconds": round(ext, 1), "probe_tuples_per_s": round((1 << 28) / ext, 2),
                                           "note": "quadratic extrapolation from the measured sample, not measured"}})

    head = v2(log2n, 100, allc)                      # the headline: reference ratio, all cores
    v2(max(16, log2n - 2), 100, 1)                   # 1 core (bounded sample)
    v2(log2n, 1, allc)                               # H = |R|
    v2(log2n, 1, 1)
    nested(17, allc)
    nested(16, 1)
    if O.ref_available():
        ref_nested(16)
    return {"value": head["probe_tuples_per_s"], "unit": "probe tuples/s", "cores": allc, "kind": "port",
            "sample": f"join_v2 restated (oracle/hj_oracle.c), |R|=|S|=2^{log2n} PK-FK int64, H=|R|/100 "
                      f"(reference ratio), {allc} host threads; probe = count + probe phases "
                      f"({head['phases_s']['count'] + head['phases_s']['probe']:.2f} s)",
            "host": facts, "runs": runs}


# ---------------------------------------------------------------- roofline helpers
def kernel_source_sha():
    h = hashlib.sha256()
    for f in ("hj_radix.hip", "hj_kernels.hip", "hj_internal.h", "hj_gen.h"):
        with open(os.path.join(ROOT, "mlir-hashjoin_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_record(config, n_gpus):
    """This workload's rocprofv3 PMC summary (profiles/pmc_latest.json, written
    by profiles/pmc_to_json.py) if it was collected from the current kernel
    sources, else (None, reason)."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_latest.json"
    e = d.get(f"{config}/n{n_gpus}")
    if not e:
        return None, f"no PMC record for {config}/n{n_gpus}"
    if e.get("source_sha") != kernel_source_sha():
        return None, f"stale: PMC of kernel sources {e.get('source_sha')} (now {kernel_source_sha()})"
    return e, f"rocprofv3 PMC, {e.get('source', '')}"


def traffic_of(rec, names, optional=(), pass_forms=None):
    """HBM bytes per launch summed over the probe phase's kernels (and those
    of `optional` that ran).  pass_forms: the k_pass variants of the phase
    (substring of the template arguments, e.g. "true, 4," for the bucketed
    second pass); default every variant."""
    if not rec:
        return None
    ks = rec.get("kernels", {})
    tot = 0
    for base in tuple(names) + tuple(b for b in optional if b in ks):
        k = ks.get(base)
        if not k:
            return None
        if base == "k_pass":
            # the S side runs each k_pass variant once: sum the variants' averages
            vs = [v for name, v in k["variants"].items() if pass_forms is None or any(f in name for f in pass_forms)]
            if not vs:
                return None
            tot += sum(v["hbm_bytes_per_launch"] for v in vs)
        else:
            tot += k["hbm_bytes_per_launch"]
    return int(tot)


def copy_floor(hashjoin, reps=5):
    """This box's streamed-copy rate, measured in-process: 2^28 16-B rows
    (4 GiB read + 4 GiB written) copied by hj_dev_stream_copy in the radix
    passes' persistent shape and in the flat one-row-per-thread shape; HIP
    events on the launching stream, median of `reps`."""
    rows = COPY_FLOOR_ROWS
    a = torch.full((2 * rows,), 7, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    nbytes = 2 * rows * 16
    res = {"bytes": nbytes, "reps": reps}
    for shape in ("persistent", "flat"):
        hashjoin.stream_copy(a, b, shape)
        ts = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            hashjoin.stream_copy(a, b, shape)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        med = ts[len(ts) // 2]
        res[f"{shape}_ms"] = round(med, 4)
        res[f"{shape}_gbs"] = round(nbytes / (med / 1000.0) / 1e9, 1)
    assert bool((b[:4] == 7).all()), "copy floor: destination not written"
    del a, b
    torch.cuda.empty_cache()
    res["shapes"] = ("persistent: one 1024-thread workgroup per CU, contiguous 4096-row tile range, next tile "
                     "prefetched (the passes' shape); flat: one row per thread, 256-thread workgroups; nt loads "
                     "and stores")
    return res


# ---------------------------------------------------------------- main
def gen_inputs(hashjoin, a, NR, NS, distn, r0, nr, s0, ns):
    if distn == "pkfk":
        return hashjoin.gen_pkfk(a.seed, NR, NS, 1.0, r0, nr, s0, ns)
    if distn == "zipf":
        rk, rp, _, _ = hashjoin.gen_pkfk(a.seed, NR, NS, 1.0, r0, nr, s0, 0)
        sk, sp = hashjoin.gen_zipf(a.seed, NR, NS, 0.9, s0, ns)
        return rk, rp, sk, sp
    if distn == "ref100k64":
        rk, rp = hashjoin.gen_uniform_i64(a.seed, 1, 1, 100_000, nr, i0=r0)
        sk, sp = hashjoin.gen_uniform_i64(a.seed, 2, 1, 100_000, ns, i0=s0)
        return rk, rp, sk, sp
    if distn == "uniform30":
        rk, rp = hashjoin.gen_uniform_i64(a.seed, 1, 1, 1 << 30, nr, i0=r0)
        sk, sp = hashjoin.gen_uniform_i64(a.seed, 2, 1, 1 << 30, ns, i0=s0)
        return rk, rp, sk, sp
    hi = 100_000 if distn == "ref100k" else 1_000_000_000
    return (hashjoin.gen_uniform_i32(a.seed, 1, 1, hi, nr, i0=r0), None,
            hashjoin.gen_uniform_i32(a.seed, 2, 1, hi, ns, i0=s0), None)


def expected_rows(distn, NR, NS):
    return NS if distn in ("pkfk", "zipf") else None


def host_leg(hashjoin, seed):
    """The literal drop-in: hj_count_i64 -> hj_probe_i64 over HOST memrefs
    (run_test.sh's call shape), PCIe included, 2^24 x 2^24 PK-FK int64."""
    import numpy as np
    from hashjoin import memref as MR
    n = 1 << 24
    rk, rp, sk, sp = (t.cpu().numpy() for t in hashjoin.gen_pkfk(seed, n, n))
    MR.count_i64(rk[:1024], rp[:1024], sk[:1024], sp[:1024])   # warm
    h0 = hashjoin.lib.hj_host_memo_hits()
    t0 = time.perf_counter()
    m = MR.count_i64(rk, rp, sk, sp)
    t1 = time.perf_counter()
    o_r = np.empty(m, np.int64)
    o_s = np.empty(m, np.int64)
    rc = MR.probe_i64(rk, rp, sk, sp, o_r, o_s)
    t2 = time.perf_counter()
    assert rc == 0 and m == n
    # the output download alone: M rows x two int64 columns, device -> fresh
    # host arrays (what the probe must at least spend after the count)
    import torch
    d = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(2)]
    h = [np.empty(m, np.int64) for _ in range(2)]
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for x, y in zip(d, h):
        torch.from_numpy(y).copy_(x)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    return {"api": "hj_count_i64 -> hj_probe_i64 (host memrefs, PCIe Gen5 included)", "rows": "2^24 x 2^24",
            "count_ms": round((t1 - t0) * 1e3, 2), "probe_ms": round((t2 - t1) * 1e3, 2),
            "download_ms": round((t4 - t3) * 1e3, 2),
            "probe_reused_count_join": hashjoin.lib.hj_host_memo_hits() == h0 + 1,
            "probe_tuples_per_s_end_to_end": round(n / (t2 - t0), 1),
            "pcie_payload_bytes": n * 32 * 2 + m * 16}


def main():
    a = parse()
    # stdout carries exactly ONE JSON line: everything else written to fd 1
    # (RCCL's init banner, library chatter) goes to stderr instead
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
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

    NR, NS, distn, ktype, desc = CONFIGS[a.config]
    if a.log2:
        NR = NS = 1 << a.log2
        desc = f"{desc} (resized: |R|=|S|=2^{a.log2})"
    wide = ktype == "int64"
    if use_dist and not wide:
        raise SystemExit("the multi-GPU path joins int64 key/payload columns")
    r0, nr = rank * NR // world, (rank + 1) * NR // world - rank * NR // world
    s0, ns = rank * NS // world, (rank + 1) * NS // world - rank * NS // world
    rk, rp, sk, sp = gen_inputs(hashjoin, a, NR, NS, distn, r0, nr, s0, ns)
    hj = hashjoin.HashJoin(local)
    hj.set_strategy(a.strategy, radix_bits=a.radix_bits)
    expect_m = expected_rows(distn, NR, NS)
    torch.cuda.synchronize()

    phases = {"init": 0.0, "build": 0.0, "probe": 0.0, "probe_partition": 0.0, "probe_join": 0.0, "route": 0.0,
              "s_route": 0.0}
    last = {}

    if not use_dist:
        hj.allocate_hash_table(NR, 64 if wide else 32)
        hj.build_table(rk, rp)
        hj.reserve_probe(NS, 64 if wide else 32)
        odt = torch.int64 if wide else torch.int32
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        # size the output once: the exact M (a count) for the duplicate-heavy
        # workloads, |S| for the key joins
        if expect_m is None:
            hj.probe_relation(sk, sp, None, None, count=cnt)
            cap = int(cnt.item())
        else:
            cap = NS
        out_r = torch.empty(max(cap, 1), dtype=odt, device="cuda")
        out_s = torch.empty_like(out_r)
        # phase times from HIP events recorded inside every step, summed
        # after the steps (hj_ctx_timing_accumulate): the steps run back to
        # back with no host synchronisation between them; M (cnt) is read
        # once the timed steps are over
        hj.accumulate_timing(True)

        def step(acc):
            hj.build_table(rk, rp)
            hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    else:
        # strong scaling over the GLOBAL relations; output stays distributed
        hj.allocate_hash_table(2 * nr, 64)

        def step(acc):
            ev = {}
            o_r, o_s = distributed_join(hj, rk, rp, sk, sp, phases=ev, n_build_global=NR,
                                        s_parts=a.s_parts or None)
            ev["probed"].synchronize()
            if acc:
                # transfers overlap compute (hashjoin.dist): R's tuples move
                # during S's routing, S's during R's build
                phases["route"] += ev["start"].elapsed_time(ev["routed"])
                if "s_route" in ev:
                    phases["s_route"] += ev["s_route"].elapsed_time(ev["routed"])
                phases["build"] += ev["routed"].elapsed_time(ev["built"])
                phases["probe"] += ev["built"].elapsed_time(ev["probed"])
            last["m"] = o_r.numel()
            last["rows"] = ev["rows"]
            last["mode"] = ev["mode"] + (", folded routing" if ev.get("folded") else "")

    # the box's own copy rate (outside the timed steps): every line states how
    # far its probe phase is from it (roofline.floor_ms / phase_over_floor)
    floor = None if a.no_floor else copy_floor(hashjoin)
    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if not use_dist:
        hj.timing_totals()   # (drops the warmup steps' times)
    if use_dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not use_dist:
        tot = hj.timing_totals()
        if tot["steps"] != a.steps:
            raise SystemExit(f"timing covered {tot['steps']} steps, expected {a.steps}")
        for k in ("init", "build", "probe", "probe_partition", "probe_join"):
            phases[k] += max(0.0, tot[k])
        last["m"] = int(cnt.item())

    m_local = last["m"]
    per_rank = None
    if use_dist:
        mine = torch.tensor([elapsed, float(m_local), float(last["rows"][0]), float(last["rows"][1]),
                             phases["route"] / a.steps, phases["build"] / a.steps, phases["probe"] / a.steps],
                            dtype=torch.float64, device="cuda")
        allr = torch.empty(world * mine.numel(), dtype=torch.float64, device="cuda")
        dist.all_gather_into_tensor(allr, mine)
        allr = allr.view(world, -1).cpu().tolist()
        elapsed = max(r[0] for r in allr)
        m_total = int(sum(r[1] for r in allr))
        per_rank = [{"rank": i, "result_rows": int(r[1]), "build_rows": int(r[2]), "probe_rows": int(r[3]),
                     "route_ms": round(r[4], 4), "build_ms": round(r[5], 4), "probe_ms": round(r[6], 4),
                     "ms_per_step": round(r[0] * 1e3 / a.steps, 4)} for i, r in enumerate(allr)]
    else:
        m_total = m_local
    if expect_m is not None and m_total != expect_m:
        raise SystemExit(f"join produced {m_total} rows, expected {expect_m}")

    if a.verify and not use_dist:
        o_r, o_s = out_r[:m_local].long(), out_s[:m_local].long()
        assert bool((rk[o_r] == sk[o_s]).all()), "non-matching pair in output"

    ms = elapsed * 1000.0 / a.steps
    value = NS / (ms / 1000.0)
    ph = {k: round(v / a.steps, 4) for k, v in phases.items() if v > 0}

    # SURVEY 8(d) algorithmic bytes.  int64: 16 B S row + 16 B slot + 16 B
    # output pair per probe row (48 B at f = 1); i32 (reference types): 4 B
    # S key + 8 B slot + 8 B output pair.
    K, SLOT, PAIR = (16, 16, 16) if wide else (4, 8, 8)
    probe_ms = phases["probe"] / a.steps
    join_ms = phases["probe_join"] / a.steps
    build_ms = (phases["init"] + phases["build"]) / a.steps
    strategy = hj.strategy_used or a.strategy
    probe_bytes = ns * (K + SLOT) + m_local * PAIR
    read_bytes = ns * (K + SLOT)
    if use_dist:
        nr_loc, ns_loc = last["rows"]
        probe_bytes = ns_loc * (K + SLOT) + m_local * PAIR
        read_bytes = ns_loc * (K + SLOT)
    rec, traffic_note = pmc_record(a.config + ("-dist" if use_dist else ""), world)
    info = hashjoin.device_info(local)

    s_route_ms = phases["s_route"] / a.steps
    # structural HBM bytes of t_probe: every S partition pass + the join
    W = 16 if wide else 8
    kbytes_loc = ((last["rows"][0] if use_dist else nr) + (last["rows"][1] if use_dist else ns)) * W + m_local * PAIR
    ns_probe = last["rows"][1] if use_dist else ns
    if use_dist and s_route_ms > 0:
        # S: key histogram (8 B) + EXACT pass (32 B) in the route, one local pass (32 B)
        structure = ns * (8 + 32) + ns_probe * 32 + kbytes_loc
    elif wide:
        structure = ns_probe * 32 * max(1, hj.radix_passes) + kbytes_loc
    else:
        structure = ns_probe * (12 + 16 * max(0, hj.radix_passes - 1)) + kbytes_loc
    roof = probe_roofline(strategy, use_dist, probe_ms, s_route_ms, probe_bytes, read_bytes,
                          structure_bytes=structure if strategy == "radix" else None, floor=floor)
    roof["bytes_per_probe_row"] = round(probe_bytes / max(1, ns if not use_dist else last["rows"][1]), 2)
    if strategy == "radix" and use_dist and world == 1 and "local_probe" in roof:
        # every S kernel of t_probe: EXACT + local k_pass variants, the key histogram, the join
        roof["traffic"] = traffic_of(rec, PROBE_KERNELS, OPTIONAL_PROBE_KERNELS + ("k_slot_hist",))
        roof["local_probe"]["traffic"] = traffic_of(rec, PROBE_KERNELS, OPTIONAL_PROBE_KERNELS,
                                                    pass_forms=("<true, 4,", "<false, 4,"))
    elif strategy == "radix" and not use_dist:
        roof["traffic"] = traffic_of(rec, PROBE_KERNELS, OPTIONAL_PROBE_KERNELS)
    else:
        roof["traffic"] = None
    roof["traffic_source"] = traffic_note
    if floor:
        roof["copy_floor"] = floor
    frac = frac_of
    if not use_dist and strategy == "radix":
        kbytes = (nr + ns) * (16 if wide else 8) + m_local * PAIR
        # the kernel is a function of the data (row width, |S| / |R|, the build
        # side's sampled repeats), reported by the context itself
        kname = hj.join_kernel or "?"
        kbase = kname.replace("_stream", "")
        ran = [kbase] if rec and kbase in rec.get("kernels", {}) else []
        roof["kernel"] = {"name": kname + " (hj_radix.hip; + k_join over deferred items)",
                          "achieved": round(kbytes / (join_ms / 1000.0) / 1e9, 1)
                          if join_ms > 0 else None, "frac": frac(kbytes, join_ms),
                          "algorithmic_bytes_per_launch": kbytes, "avg_launch_ms": round(join_ms, 4),
                          "traffic": traffic_of(rec, (), ran) if ran else None}
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
        "dtype": ktype,
        "data": f"synthetic (counter-based generator, seed {a.seed:#x}, generated on device)",
        "config": {"workload": f"{a.config}: {desc}", "R_rows": NR, "S_rows": NS, "key": ktype,
                   "payload": "int64" if wide else "row id (i32)", "distribution": distn,
                   "parallelism": ("single GPU" if not use_dist
                                   else f"hash-routed x{world} ({last['mode']}), RCCL")},
        "joined_rows_per_sec": round(m_total / (ms / 1000.0), 1),
        "result_rows": m_total,
        "phase_ms": ph,
        "strategy": strategy,
        "roofline": roof,
        "build_phase": {
            "kernel": f"k_pass x{hj.radix_passes}" if strategy == "radix" else "k_init + k_build",
            "algorithmic_bytes": nr * 32 * max(1, hj.radix_passes if strategy == "radix" else 1),
            "ms": round(build_ms, 4),
        },
        # the bucket sets' row buffers, probed and redrawn at allocation
        # (hj_placement_stats; done in the untimed first call)
        "placement": hashjoin.placement_stats(),
        "device": {"name": torch.cuda.get_device_name(local), **info,
                   "peak_used_gbs": HBM_PEAK_GBS,
                   "peak_note": "8.0 TB/s spec (MI355X_MICROARCH.md); peak_mb_per_s = hipDeviceProp "
                                "memoryBusWidth/8 x memoryClockRate x 4 (HBM3E transfers per reported clock)"},
    }
    if a.config in REFERENCE_PUBLISHED:
        pub = REFERENCE_PUBLISHED[a.config]
        line["reference_published"] = {**pub, "probe_tuples_per_s_join_v2": round(NS / pub["join_v2_s"], 1),
                                       "speedup_vs_join_v2": round(value / (NS / pub["join_v2_s"]), 1),
                                       "note": "reference on sm_86 with module loads in its timers; a "
                                               "different GPU, not a like-for-like baseline"}
    if per_rank is not None:
        line["per_rank"] = per_rank
    if rank == 0 and not use_dist and not a.no_host_leg and a.config == "C3":
        line["host_memref"] = host_leg(hashjoin, a.seed)
    if rank == 0 and not use_dist and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(a.seed, a.cpu_sample_log2)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    hj.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
