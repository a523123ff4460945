"""Summarise tools/chunk_handoff.sh: per step, the S pass-2 and join kernel time
of the chunked probe, interleaved (hand-off) against split (no hand-off).

Usage: python tools/chunk_summary.py gpurun_out/handoff
"""
import csv
import glob
import json
import os
import sys


def kernels(path):
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        name = r["Kernel_Name"].replace("hj::(anonymous namespace)::", "")
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    out.sort()
    return out


def summarise(trace):
    ks = kernels(trace)
    # segments between first passes (k_pass<true, 0 ...>); a probe's segment holds its joins
    p1 = [i for i, k in enumerate(ks) if k[2].startswith("void k_pass<true, 0")] + [len(ks)]
    steps = []
    for a, b in zip(p1, p1[1:]):
        seg = ks[a:b]
        njoin = sum(1 for k in seg if k[2].startswith("void k_join_b"))
        if njoin == 0:
            continue
        tot = lambda pred: sum(k[1] - k[0] for k in seg if pred(k[2])) / 1e6
        pass2 = tot(lambda n: n.startswith("void k_pass<true, 4"))
        joinb = tot(lambda n: n.startswith("void k_join_b"))
        small = tot(lambda n: not n.startswith("void k_pass") and not n.startswith("void k_join_b"))
        steps.append((pass2, joinb, small, njoin))
    steps = steps[1:] if len(steps) > 1 else steps   # drop the warmup step
    n = len(steps)
    return tuple(sum(s[i] for s in steps) / n for i in range(3)) + (steps[0][3],)


def main(d):
    print(f"{'run':<14} {'chunks':>6} {'S pass2 ms':>10} {'join_b ms':>10} {'small ms':>9} {'probe ms':>9}")
    for t in sorted(glob.glob(os.path.join(d, "*", "t_kernel_trace.csv"))):
        run = os.path.basename(os.path.dirname(t))
        pass2, joinb, small, nj = summarise(t)
        js = os.path.join(d, run + ".json")
        probe = json.load(open(js))["phase_ms"]["probe"] if os.path.exists(js) else float("nan")
        print(f"{run:<14} {nj:>6} {pass2:10.3f} {joinb:10.3f} {small:9.3f} {probe:9.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/handoff")
