#!/bin/bash
# k_join_b ballot stores plain (build/plainb) vs non-temporal (product): A/B + write bytes
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06m}
cd $R && mkdir -p gpurun_out/$TAG
bash tools/ab_alt.sh $TAG "C3 REF-B C1-ref" plainb 2 || exit 1
cd /tmp && export TMPDIR=/tmp
for C in C3 REF-B; do
  for V in plainb product; do
    if [ $V = product ]; then L=$R/mlir-hashjoin_amd/lib/libhj.so; else L=$R/build/$V/libhj.so; fi
    HJ_LIB=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/${V}_${C}_W -o run -- python3 $R/bench.py --config $C --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > $R/gpurun_out/$TAG/${V}_${C}_W.log 2>&1 || { echo "pmc $V $C rc=$?"; exit 1; }
    python3 - $R/gpurun_out/$TAG/${V}_${C}_W $V $C <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
v = sorted(float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_join_b<" in r["Kernel_Name"] and ("<true, true" in r["Kernel_Name"] or "<false, true" in r["Kernel_Name"]))
print(sys.argv[2], sys.argv[3], "k_join_b WRITE_SIZE median GB %.4f (n=%d)" % (v[len(v) // 2] * 1024 / 1e9, len(v)))
PY
  done
done
