#!/bin/bash
# join R-prefetch placement: product = one prefetch site at the item's end (B), vs base (none) and A (after the first scan)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05o
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05o/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05o/tests.log; exit 1; }
tail -1 gpurun_out/r05o/tests.log
bash tools/ab_alt.sh r05o_base "C3 REF-B C1-ref" base 2 && bash tools/ab_alt.sh r05o_A "C3 REF-B C1-ref" pfA 2
