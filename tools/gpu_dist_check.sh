#!/bin/bash
# GPU check of the multi-GPU code paths on one GPU: dist tests (world-1 RCCL,
# owner splits, folded routing) and the forced-distributed C3 bench line.
#   tools/gpu_dist_check.sh <tag>
set -o pipefail
TAG=$1
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/${TAG}_dist.log 2>&1 || { tail -40 gpurun_out/${TAG}_dist.log; exit 1; }
tail -2 gpurun_out/${TAG}_dist.log
timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    > gpurun_out/${TAG}_fd.json 2> gpurun_out/${TAG}_fd.err || { tail gpurun_out/${TAG}_fd.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_fd.json')); print(d['ms_per_step'], d['phase_ms'], d.get('per_rank'))"
