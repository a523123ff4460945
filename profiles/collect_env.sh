#!/bin/bash
# Like collect.sh but only the kernel-trace + L2 hit + FETCH/WRITE passes,
# for A/B runs under an environment override:  collect_env.sh <tag> <VAR=val> [bench args...]
set -euo pipefail
TAG=$1; shift
ENVSET=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export "$ENVSET"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$N" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/pmc_$N.log" 2>&1
done
echo done > "$OUT/DONE"
