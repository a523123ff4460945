#!/bin/bash
# join launch merge: the GPU tests that cover kernel choice / deferrals, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_skew.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05f/tests.log; exit 1; }
tail -2 gpurun_out/r05f/tests.log
bash tools/ab_alt.sh r05f "C3 REF-A64 REF-A REF-B" base 2
