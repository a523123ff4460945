#!/bin/bash
# A/B bench lines of experiment builds (build/<variant>/libhj.so, made with
#   make -C mlir-hashjoin_amd OUT=$PWD/build/<variant> EXTRA=-D...)
# against the product library:  tools/ab_libs.sh <tag> "<configs>" <variant>...
set -o pipefail
TAG=$1; CONFIGS=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.jsonl
for V in product "$@"; do
  for C in $CONFIGS; do
    if [ "$V" = product ]; then LIB=$R/mlir-hashjoin_amd/lib/libhj.so; else LIB=$R/build/$V/libhj.so; fi
    HJ_LIB=$LIB timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
        > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}_ab.err || { echo "BENCH $V $C FAILED"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_one.json')); d['variant']='$V'; print(json.dumps(d))" >> $OUT
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_one.json')); p=d['phase_ms']; print('$V', '$C', d['ms_per_step'], 'join', p.get('probe_join'), 'probe', p.get('probe'), d['roofline'].get('kernel',{}).get('name','')[:12])"
  done
done
