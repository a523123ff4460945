#!/bin/bash
# k_join_b: run-edge sectors plain, the rest non-temporal (build/e32, e64,
# e128 = -DHJ_EDGE_B) vs the product (all nt): alternating A/B + C3 write bytes
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06r}
cd $R && mkdir -p gpurun_out/$TAG
bash tools/ab_alt.sh $TAG "C3 C1 C1-ref REF-B" "e32 e64 e128" 2 || exit 1
cd /tmp && export TMPDIR=/tmp
for V in e32 e64 e128 product; do
  if [ $V = product ]; then L=$R/mlir-hashjoin_amd/lib/libhj.so; else L=$R/build/$V/libhj.so; fi
  HJ_LIB=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/${V}_C3_W -o run -- python3 $R/bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > $R/gpurun_out/$TAG/${V}_C3_W.log 2>&1 || { echo "pmc $V rc=$?"; exit 1; }
  python3 - $R/gpurun_out/$TAG/${V}_C3_W $V <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
v = sorted(float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_join_b<true, true" in r["Kernel_Name"])
print(sys.argv[2], "C3 k_join_b WRITE_SIZE median GB %.4f (n=%d)" % (v[len(v) // 2] * 1024 / 1e9, len(v)))
PY
done
