#!/bin/bash
# bench line per config (no CPU baseline / host leg) + the forced-distributed C3 line and its kernel trace
#   tools/r05x_sweep.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
for C in C3 C1 C1-ref C2 C4 REF-A REF-B REF-A64; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/$TAG/bench.jsonl 2>> gpurun_out/$TAG/bench.err || { echo "BENCH $C FAILED"; exit 1; }
done
timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    >> gpurun_out/$TAG/bench.jsonl 2>> gpurun_out/$TAG/bench.err || { echo "BENCH dist FAILED"; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/$TAG/bench.jsonl'):
    d=json.loads(l); r=d['roofline']
    print(d['config']['workload'][:8], d['ms_per_step'], 'frac', r.get('frac'), {k:round(v,3) for k,v in d['phase_ms'].items() if v}, d.get('placement',{}).get('rejected'))
"


cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace_dist -o run -- \
    python3 $R/bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $R/gpurun_out/$TAG/trace_dist.log 2>&1 || echo "trace rc=$?"
