#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run: per-kernel average duration (kernel
trace) and per-dispatch PMC counters, with the gfx950 byte conversions of
MI355X_MICROARCH.md ("HBM"): FETCH_SIZE reports 1/2 of a wide streaming read
(doubled here as `fetch_bytes_x2`), WRITE_SIZE is exact for 16-B-per-lane
stores; TCC_EA0_RDREQ_{32B,64B,128B} give the fabric read requests by size.

usage: summarize.py <prof_dir> [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(s):
    m = re.search(r"(k_\w+)(<[^>]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:60]


def main():
    d = sys.argv[1]
    out = {"kernels": {}}
    ks = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(ks):
        for row in csv.DictReader(open(ks)):
            k = kname(row["Name"])
            out["kernels"].setdefault(k, {})["avg_ns"] = float(row["AverageNs"])
            out["kernels"][k]["calls"] = int(row["Calls"])
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(list)
        for row in csv.DictReader(open(f)):
            agg[(kname(row["Kernel_Name"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
        for (k, c), v in agg.items():
            out["kernels"].setdefault(k, {})[c] = sum(v) / len(v)
    for k, e in out["kernels"].items():
        if "FETCH_SIZE" in e:
            e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in e:
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
        if "TCC_EA0_RDREQ_sum" in e:
            r32 = e.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            e["rdreq_bytes_est"] = (e["TCC_EA0_RDREQ_sum"] - r32) * 64 + r32 * 32
        if "TCC_EA0_WRREQ_sum" in e:
            w64 = e.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            e["wrreq_bytes_est"] = w64 * 64 + (e["TCC_EA0_WRREQ_sum"] - w64) * 32
    for k, e in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("avg_ns", 0)):
        if not k.startswith("k_"):
            continue
        t = e.get("avg_ns", 0) / 1e6
        fields = [f"{k:34s}", f"{t:9.3f} ms"]
        for c in ("fetch_bytes_x2", "write_bytes", "rdreq_bytes_est", "wrreq_bytes_est"):
            if c in e:
                fields.append(f"{c}={e[c] / 1e9:.3f} GB")
        if "TCC_HIT_sum" in e:
            h, m = e["TCC_HIT_sum"], e.get("TCC_MISS_sum", 0)
            fields.append(f"L2hit={h / max(1, h + m):.3f}")
        print("  ".join(fields))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
