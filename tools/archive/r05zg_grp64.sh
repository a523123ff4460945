#!/bin/bash
# grouped join for int64 rows: tests (radix, parity, dist, reference workloads), then A/B vs the previous commit
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05zg
timeout -k 10 900 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_reference_workloads.py tests/test_gpu_rows.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zg/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05zg/tests.log; exit 1; }
tail -1 gpurun_out/r05zg/tests.log
bash tools/ab_alt.sh r05zg "REF-A64 C3 REF-A" base5 2
