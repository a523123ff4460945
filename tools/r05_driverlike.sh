#!/bin/bash
# the round-end driver's order on a fresh box: GPU suite, smoke(), then the bench command
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05_final}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1 || { tail -20 gpurun_out/$TAG/gputest.log; exit 1; }
tail -1 gpurun_out/$TAG/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); r=d['roofline']
print(d['ms_per_step'], d['value'], d['phase_ms'], 'frac', r['frac'], 'traffic', r.get('traffic'), 'floor', r.get('floor_ms'), r.get('phase_over_floor'), 'placement', d['placement']['probes'], d['placement']['rejected'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))
"
