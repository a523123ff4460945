#!/bin/bash
# k_join_b (int64 rows): the next item's descriptor staged through LDS one
# item ahead (build/da = -DHJ_DESC_AHEAD=1) vs the product: parity + A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06s}
V=${2:-da}
cd $R && mkdir -p gpurun_out/$TAG
HJ_LIB=$R/build/$V/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests_$V.log 2>&1 || { echo TESTS $V FAILED; tail -30 gpurun_out/$TAG/tests_$V.log; exit 1; }
tail -1 gpurun_out/$TAG/tests_$V.log
bash tools/ab_alt.sh $TAG "C3 C4 C1 C1-ref" "$V" 2
