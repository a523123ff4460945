#!/bin/bash
# Round 6 final: the driver's order on a fresh box (GPU suite, smoke(), the
# default bench command), then every config's bench line (one box)
#   tools/r06/final_driver.sh <tag> [sweep]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06_final}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1 || { tail -30 gpurun_out/$TAG/gputest.log; exit 1; }
tail -1 gpurun_out/$TAG/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); r=d['roofline']
print(d['ms_per_step'], d['value'], d['phase_ms'], 'frac', r['frac'], 'traffic', r.get('traffic'), 'floor', r.get('floor_ms'), r.get('phase_over_floor'), r.get('phase_over_flat_floor'), 'placement', d['placement'])
"
if [ "${2:-}" = sweep ]; then
  for C in C3 C1 C1-ref C2 C4 REF-A REF-B REF-A64; do
    timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
        >> gpurun_out/$TAG/sweep.jsonl 2>> gpurun_out/$TAG/sweep.err || { echo "BENCH $C FAILED"; exit 1; }
    tail -1 gpurun_out/$TAG/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'].get('workload','')[:40], d['ms_per_step'], d['phase_ms'], d['roofline'].get('frac'))"
  done
  timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/$TAG/sweep.jsonl 2>> gpurun_out/$TAG/sweep.err || { echo "BENCH forced-dist FAILED"; exit 1; }
  tail -1 gpurun_out/$TAG/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 forced-dist', d['ms_per_step'], d['phase_ms'])"
fi
