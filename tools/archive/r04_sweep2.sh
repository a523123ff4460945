#!/bin/bash
# round-4: a second box's bench lines of the final kernels (every config +
# forced-dist), then an A/B of experiment builds
#   tools/r04_sweep2.sh <tag> "<ab configs>" <variant> ...
set -o pipefail
TAG=$1; ABC=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for C in C3 C1 C1-ref C2 C4 REF-A REF-B; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH $C FAILED"; exit 1; }
done
timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH forced-dist FAILED"; exit 1; }
echo sweep done
[ $# -gt 0 ] && bash tools/ab_libs.sh ${TAG} "$ABC" "$@"
exit 0
