#!/bin/bash
# placement probe: GPU tests of the radix path, then ten fresh contexts off / on / off / on
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05v/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05v/tests.log; exit 1; }
tail -1 gpurun_out/r05v/tests.log
for k in 1 2; do
  HJ_PLACEMENT_PROBE=0 timeout -k 10 300 python -u tools/xp_place.py 10 >> gpurun_out/r05v/ab.jsonl 2>> gpurun_out/r05v/ab.err || { tail -5 gpurun_out/r05v/ab.err; exit 1; }
  timeout -k 10 300 python -u tools/xp_place.py 10 >> gpurun_out/r05v/ab.jsonl 2>> gpurun_out/r05v/ab.err || { tail -5 gpurun_out/r05v/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/r05v/ab.jsonl'):
    d=json.loads(l); print(d['probe_env'], d['ctx'], d['build'], d['probe_partition'], d['probe_join'], d['placement'])
"
