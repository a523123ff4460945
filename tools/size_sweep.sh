#!/bin/bash
# Per-row cost of the join and the partition passes against the relation size
# (PK-FK, |R| = |S| = 2^k): where the working set fits the Infinity Cache the
# join's loads are served on-die.  One JSON line per size into $OUT/sweep.jsonl.
set -uo pipefail
TAG=${1:-size_sweep}; shift || true
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for K in ${SIZES:-20 21 22 23 24 26 28}; do
  timeout -k 10 120 python3 bench.py --config C1 --log2 $K --no-cpu-baseline --no-host-leg --steps 10 "$@" \
      > "$OUT/k$K.json" 2> "$OUT/k$K.err" || exit 1
  python3 - "$OUT/k$K.json" $K <<'PY' | tee -a "$OUT/sweep.txt"
import json, sys
d = json.load(open(sys.argv[1])); k = int(sys.argv[2]); n = 1 << k; p = d["phase_ms"]
print(f"2^{k:2d}  step {d['ms_per_step']:7.3f} ms  build {p['build']:6.3f}  S-part {p['probe_partition']:6.3f}"
      f"  join {p['probe_join']:6.3f} ms  join ps/row {p['probe_join']*1e9/n:6.2f}  S-part ps/row {p['probe_partition']*1e9/n:6.2f}")
PY
done
echo SWEEP_DONE
