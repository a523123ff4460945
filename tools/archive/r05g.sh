#!/bin/bash
# fused small-pass listing scan: tests, a C3 trace (launches per step), A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05g; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-leg --no-floor --steps 5 --warmup 2 > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
cd $R && bash tools/ab_alt.sh r05g "C3 C1" base 2
