#!/bin/bash
# bucket sizes again with the placement probe: final sets 1024-row buckets (f10), intermediate 2048 (p11)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05zd
for V in f10 p11; do
  HJ_LIB=$R/build/$V/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zd/tests_$V.log 2>&1 || { echo TESTS $V FAILED; tail -20 gpurun_out/r05zd/tests_$V.log; exit 1; }
  tail -1 gpurun_out/r05zd/tests_$V.log
done
bash tools/ab_alt.sh r05zd_f "C3 C4" f10 2 && bash tools/ab_alt.sh r05zd_p "C3 C4" p11 2
