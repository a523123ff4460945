#!/bin/bash
# Bench sweep on one MI355X (run through gpurun): every BASELINE config and
# the reference workloads, one JSON line each into gpurun_out/$TAG/bench.jsonl.
set -uo pipefail
TAG=${1:-sweep}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --config C3 > "$OUT/c3.json" 2> "$OUT/c3.err" || exit 1
cat "$OUT/c3.json" >> "$OUT/bench.jsonl"
for C in C1 C1-ref C2 C4 REF-A REF-B; do
  timeout -k 10 200 python3 bench.py --config $C --no-cpu-baseline > "$OUT/$C.json" 2> "$OUT/$C.err" || exit 1
  cat "$OUT/$C.json" >> "$OUT/bench.jsonl"
done
timeout -k 10 200 python3 bench.py --config C3 --force-dist --no-cpu-baseline > "$OUT/c3_dist1.json" 2> "$OUT/c3_dist1.err" || exit 1
cat "$OUT/c3_dist1.json" >> "$OUT/bench.jsonl"
echo SWEEP_DONE
