#!/bin/bash
# Quick join check on one MI355X (gpurun): radix/parity GPU tests, then one
# bench line per config.  usage: tools/join_check.sh TAG "CONFIGS" [extra bench args]
set -uo pipefail
TAG=$1; CONFIGS=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for C in $CONFIGS; do
  timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-host-leg "$@" > "$OUT/$C.json" 2> "$OUT/$C.err" || { echo "BENCH FAIL $C"; exit 1; }
  python3 -c "import json; L=open('$OUT/$C.json').read().splitlines(); d=json.loads(L[-1]); p=d['phase_ms']; print('$C', len(L), 'line(s)', d['ms_per_step'], 'S-part', p.get('probe_partition'), 'join', p.get('probe_join'))"
done
