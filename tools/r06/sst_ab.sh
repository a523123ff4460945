#!/bin/bash
# k_pass with static line stores (buffer stores, -DHJ_PASS_SST=1 = build/sst):
# pass micros, parity suites on the variant, alternating A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06sst}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 120 ./build/npass_micro > gpurun_out/$TAG/npass.txt 2>&1 || { echo NPASS FAILED; tail gpurun_out/$TAG/npass.txt; exit 1; }
head -12 gpurun_out/$TAG/npass.txt
timeout -k 10 300 ./build/pass_micro > gpurun_out/$TAG/pass.txt 2>&1 || { echo PASS FAILED; tail gpurun_out/$TAG/pass.txt; exit 1; }
grep -E "k_pass|static|pass 2 \(" gpurun_out/$TAG/pass.txt
bash tools/r06/var_ab.sh $TAG sst "${2:-C3 REF-B REF-A C1 C4}" "tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_reference_workloads.py tests/test_gpu_skew.py tests/test_gpu_dist.py" 2
