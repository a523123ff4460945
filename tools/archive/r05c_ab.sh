set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05c/tests.log; exit 1; }
tail -2 gpurun_out/r05c/tests.log
bash tools/ab_alt.sh r05c "C3 C1 REF-B C4" base 2
