#!/bin/bash
# Round 6: memory-side traffic of k_join_b, round-5 scan (old) vs per-wave claims (wave)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06g}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
for V in old wave; do
  for P in WRITE_SIZE FETCH_SIZE; do
    HJ_LIB=$R/build/$V/libhj.so timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/$TAG/${V}_$P -o run -- python3 $R/bench.py --config ${2:-C3} --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > $R/gpurun_out/$TAG/${V}_$P.log 2>&1 || { echo "pmc $V $P rc=$?"; tail -5 $R/gpurun_out/$TAG/${V}_$P.log; exit 1; }
  done
done
python3 - $R/gpurun_out/$TAG <<'PY'
import csv, sys, glob, collections
d = sys.argv[1]
for V in ["old", "wave"]:
    for P in ["WRITE_SIZE", "FETCH_SIZE"]:
        f = glob.glob(f"{d}/{V}_{P}/*counter_collection.csv")[0]
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "k_join_b" in r["Kernel_Name"] or "k_out_fixup" in r["Kernel_Name"]:
                acc[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            print(V, P, k, "calls", len(v), "median GB %.3f" % (sorted(v)[len(v) // 2] * 1024 / 1e9 if P == "WRITE_SIZE" else sorted(v)[len(v) // 2] * 2 * 1024 / 1e9))
PY
