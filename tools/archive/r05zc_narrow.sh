#!/bin/bash
# i32 join shape: 512 x 3+3 over 4096 slots at 4 workgroups per CU, partitions of <= 2048 (nB) / 1024 (nC) rows
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05zc
for V in nB nC; do
  HJ_LIB=$R/build/$V/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_reference_workloads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zc/tests_$V.log 2>&1 || { echo TESTS $V FAILED; tail -30 gpurun_out/r05zc/tests_$V.log; exit 1; }
  tail -1 gpurun_out/r05zc/tests_$V.log
done
bash tools/ab_alt.sh r05zc_B "REF-B REF-A" nB 2 && bash tools/ab_alt.sh r05zc_C "REF-B REF-A" nC 2
HJ_LIB=$R/build/wA/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_skew.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zc/tests_wA.log 2>&1 || { echo TESTS wA FAILED; tail -30 gpurun_out/r05zc/tests_wA.log; exit 1; }
tail -1 gpurun_out/r05zc/tests_wA.log
bash tools/ab_alt.sh r05zc_W "C3 C4 C1" wA 2
