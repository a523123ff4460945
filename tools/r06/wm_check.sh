#!/bin/bash
# Round 6: k_join_b wave-major output order -- join tests, A/B against
# build/old (slot-major), memory-side write bytes of both
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06h}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_reference_workloads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash tools/ab_alt.sh $TAG "C3 REF-B C1-ref" old 2 || exit 1
cd /tmp && export TMPDIR=/tmp
for C in C3 REF-B; do
  for V in old product; do
    if [ $V = product ]; then L=$R/mlir-hashjoin_amd/lib/libhj.so; else L=$R/build/$V/libhj.so; fi
    HJ_LIB=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/${V}_${C}_W -o run -- python3 $R/bench.py --config $C --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > $R/gpurun_out/$TAG/${V}_${C}_W.log 2>&1 || { echo "pmc $V $C rc=$?"; exit 1; }
    python3 - $R/gpurun_out/$TAG/${V}_${C}_W $V $C <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
v = sorted(float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_join_b" in r["Kernel_Name"] and "true, true" in r["Kernel_Name"].replace("false, true", "true, true"))
print(sys.argv[2], sys.argv[3], "k_join_b WRITE_SIZE median GB %.4f (n=%d)" % (v[len(v) // 2] * 1024 / 1e9, len(v)))
PY
  done
done
