#!/bin/bash
# join item claim issued at the item's top (stored after the build barrier): tests, A/B vs the previous commit
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05za
timeout -k 10 900 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_skew.py tests/test_gpu_reference_workloads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05za/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05za/tests.log; exit 1; }
tail -1 gpurun_out/r05za/tests.log
bash tools/ab_alt.sh r05za "C3 C4 REF-B C1-ref REF-A" base3 2
