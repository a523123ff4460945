#!/bin/bash
# k_join_b ballot stores by run (product) vs always non-temporal (build/ntb): join tests, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06n}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash tools/ab_alt.sh $TAG "${2:-C1-ref C3 REF-B C1 C4}" ntb ${3:-2} || exit 1
