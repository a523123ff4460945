#!/bin/bash
# EXPERIMENT: final sets also paired with the ping set (persistent copy tset -> fin against flat)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05ze
for k in 1 2; do
  HJ_PLACEMENT_PAIR=0 timeout -k 10 300 python -u tools/xp_place.py 8 C3 >> gpurun_out/r05ze/ab.jsonl 2>> gpurun_out/r05ze/ab.err || { tail -5 gpurun_out/r05ze/ab.err; exit 1; }
  HJ_PLACEMENT_PAIR=1 timeout -k 10 300 python -u tools/xp_place.py 8 C3 > gpurun_out/r05ze/on.jsonl 2>> gpurun_out/r05ze/ab.err || { tail -5 gpurun_out/r05ze/ab.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r05ze/on.jsonl'):
    d=json.loads(l); d['pair']=1; open('gpurun_out/r05ze/ab.jsonl','a').write(json.dumps(d)+'\n')
"
done
python3 -c "
import json
for l in open('gpurun_out/r05ze/ab.jsonl'):
    d=json.loads(l); print(d.get('pair',0), d['ctx'], d['build'], d['probe_partition'], d['probe_join'], d['placement']['probes'], d['placement']['rejected'])
"
