#!/bin/bash
# rocprofv3 collection for one bench workload (run on the GPU box via gpurun).
#   profiles/collect.sh <tag> [bench args...]
# Kernel trace + stats pass, then separate PMC passes (never combined with
# trace domains), per MI355X_MICROARCH.md "rocprofv3 PMC slots" / HBM notes.
set -euo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$N" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/pmc_$N.log" 2>&1
done
echo done > "$OUT/DONE"
