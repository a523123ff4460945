#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05s
HJ_XP_SWZ=1 HJ_LIB=build/swz/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05s/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05s/tests.log; exit 1; }
tail -1 gpurun_out/r05s/tests.log
for k in 1 2; do
HJ_XP_SWZ=0 HJ_LIB=build/swz/libhj.so timeout -k 10 300 python -u tools/xp_pad.py > gpurun_out/r05s/off$k.jsonl 2> gpurun_out/r05s/off.err || { tail -5 gpurun_out/r05s/off.err; exit 1; }
HJ_XP_SWZ=1 HJ_LIB=build/swz/libhj.so timeout -k 10 300 python -u tools/xp_pad.py > gpurun_out/r05s/on$k.jsonl 2> gpurun_out/r05s/on.err || { tail -5 gpurun_out/r05s/on.err; exit 1; }
done
for f in off1 on1 off2 on2; do echo "== $f"; python3 -c "
import json
for l in open('gpurun_out/r05s/$f.jsonl'):
    d=json.loads(l); print(d['build'], d['probe_partition'], d['probe_join'])
"; done
