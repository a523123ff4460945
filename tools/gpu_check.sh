#!/bin/bash
# GPU check used during development: GPU test suite, then bench lines.
#   tools/gpu_check.sh <tag> [config ...]     (run on the GPU box via gpurun)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
for C in "$@"; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH $C FAILED"; exit 1; }
done
python3 - "$R/gpurun_out/${TAG}_bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    r = d["roofline"]; k = r.get("kernel", {})
    print(d["config"]["workload"][:8], d["ms_per_step"], d["phase_ms"], "frac", r["frac"], "read", r.get("read_frac"),
          k.get("name"), k.get("avg_launch_ms"))
PY
