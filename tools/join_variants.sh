#!/bin/bash
# Join-kernel variant sweep on one MI355X (run through gpurun): parity tests
# under each HJ_JOIN kind, then C3 / C2 bench lines.  Output: gpurun_out/$TAG/
set -uo pipefail
TAG=${1:-jv}
KINDS=${KINDS:-"1 6 7 8"}
CONFIGS=${CONFIGS:-"C3 C2"}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for K in $KINDS; do
  if [ "${TESTS:-1}" = 1 ]; then
    HJ_JOIN=$K timeout -k 10 300 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > "$OUT/test_k$K.log" 2>&1 || { echo "TEST FAIL kind $K"; exit 1; }
    tail -1 "$OUT/test_k$K.log"
  fi
  for C in $CONFIGS; do
    HJ_JOIN=$K timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --verify \
      > "$OUT/${C}_k$K.json" 2> "$OUT/${C}_k$K.err" || { echo "BENCH FAIL $C kind $K"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${C}_k$K.json')); print('$C kind $K', d['ms_per_step'], d['phase_ms'], d.get('verify'))"
  done
done
echo SWEEP_DONE
