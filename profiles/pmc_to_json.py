#!/usr/bin/env python3
"""Record the per-launch HBM traffic of a profiles/collect.sh run in
profiles/pmc_latest.json, which bench.py reads for `roofline.traffic`.

HBM bytes per launch = FETCH_SIZE x 2 (gfx950 reports half of a wide
streaming read, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB per
dispatch, averaged over the kernel's dispatches.  Kernels are keyed by base
name (k_join, k_probe, k_pass, ...); template variants of one base name are
kept separately under "variants".

usage: pmc_to_json.py <prof_dir> <config> <n_gpus> [source-note]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    d, config, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    note = sys.argv[4] if len(sys.argv) > 4 else d
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_FETCH_SIZE", "*counter_collection.csv")) + \
            glob.glob(os.path.join(d, "pmc_WRITE_SIZE", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<[^>]*>)?", row["Kernel_Name"])
            if not m:
                continue
            per[m.group(0)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg_ns = {}
    ks = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
    if ks:
        for row in csv.DictReader(open(ks[0])):
            m = re.search(r"(k_\w+)(<[^>]*>)?", row["Name"])
            if m:
                avg_ns[m.group(0)] = float(row["AverageNs"])
    kernels = {}
    for full, c in per.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) * 1024 * 2
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) * 1024
        base = full.split("<")[0]
        e = {"hbm_bytes_per_launch": int(fetch + write), "read_bytes": int(fetch), "write_bytes": int(write),
             "avg_ms": round(avg_ns.get(full, 0.0) / 1e6, 4)}
        k = kernels.setdefault(base, {"variants": {}})
        k["variants"][full] = e
    for base, k in kernels.items():
        # the base entry is the variant with the most traffic (the hot one)
        hot = max(k["variants"].values(), key=lambda e: e["hbm_bytes_per_launch"])
        k.update(hot)
    path = os.path.join(HERE, "pmc_latest.json")
    try:
        allj = json.load(open(path))
    except (OSError, ValueError):
        allj = {}
    # the kernel sources these counters belong to: bench.py reports the
    # traffic only while they are unchanged
    sys.path.insert(0, os.path.dirname(HERE))
    from bench import kernel_source_sha
    allj[f"{config}/n{n}"] = {"source": note, "source_sha": kernel_source_sha(), "kernels": kernels}
    json.dump(allj, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(allj[f"{config}/n{n}"], indent=1))


if __name__ == "__main__":
    main()
