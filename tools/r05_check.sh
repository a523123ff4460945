#!/bin/bash
# Round 5: the whole GPU suite, then the driver's exact bench command.
#   tools/r05_check.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/$TAG/gputest.log | head; exit $rc; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err \
    || { echo "default bench failed"; tail -5 gpurun_out/$TAG/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_default.json')); r=d['roofline']; print(d['ms_per_step'], d['phase_ms'], 'frac', r['frac'], 'floor', r.get('floor_ms'), r.get('phase_over_floor'), r.get('phase_over_flat_floor'))"
