#!/bin/bash
# End-of-round check on the GPU box: GPU test suite + a bench line per config
# (tools/gpu_check.sh), the forced-distributed C3 line, then bench.py with
# its defaults (CPU baseline and host-memref leg included).
#   tools/final_sweep.sh <tag>
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
bash tools/gpu_check.sh $TAG C3 C1 C1-ref C2 C4 REF-A REF-B || exit 1
timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH forced-dist FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err \
    || { echo "DEFAULT BENCH FAILED"; tail -5 gpurun_out/${TAG}_default.err; exit 1; }
cat gpurun_out/${TAG}_default.json
