#!/bin/bash
# join: next item's first build round prefetched during the probe -- tests, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05j
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_skew.py tests/test_gpu_rows.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05j/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05j/tests.log; exit 1; }
tail -2 gpurun_out/r05j/tests.log
bash tools/ab_alt.sh r05j "C3 C4 REF-B C1-ref REF-A" base 2
