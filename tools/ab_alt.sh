#!/bin/bash
# A/B with alternating order (product, variant, product, variant, ...) so a
# drift of the box over the run does not favour whichever runs first
#   tools/ab_alt.sh <tag> "<configs>" <variant> <reps>
set -o pipefail
TAG=$1; CONFIGS=$2; V=$3; REPS=${4:-3}
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_alt.jsonl
for C in $CONFIGS; do
  for k in $(seq $REPS); do
    for W in product $V; do
      if [ "$W" = product ]; then LIB=$R/mlir-hashjoin_amd/lib/libhj.so; else LIB=$R/build/$W/libhj.so; fi
      HJ_LIB=$LIB timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
          > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}_alt.err || { echo "BENCH $W $C FAILED"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_one.json')); d['variant']='$W'; d['rep']=$k; print(json.dumps(d))" >> $OUT
      python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_one.json')); p=d['phase_ms']; print('$W', '$C', $k, d['ms_per_step'], 'build', p.get('build'), 'part', p.get('probe_partition'), 'join', p.get('probe_join'))"
    done
  done
done
