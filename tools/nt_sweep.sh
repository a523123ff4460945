#!/bin/bash
# Join load/store cache-policy sweep (HJ_NT builds in build/ntN, selected by HJ_LIB)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-nt}
mkdir -p "$OUT"; cd "$R"
for C in ${CONFIGS:-C3 C1}; do
  for V in ${VARIANTS:-prod nt0 nt4 nt8 prod}; do
    if [ "$V" = prod ]; then L=$R/mlir-hashjoin_amd/lib/libhj.so; else L=$R/build/$V/libhj.so; fi
    HJ_LIB=$L timeout -k 10 200 python bench.py --config $C --no-cpu-baseline --no-host-leg > "$OUT/${C}_$V.json" 2> "$OUT/${C}_$V.err" || exit 1
    python3 -c "import json; d=json.load(open('$OUT/${C}_$V.json')); p=d['phase_ms']; print('$C $V', d['ms_per_step'], 'join', p.get('probe_join'), 'S-part', p.get('probe_partition'))"
  done
done
echo SWEEP_DONE
