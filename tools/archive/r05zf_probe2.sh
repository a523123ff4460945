#!/bin/bash
# placement probe of the final sets in pass 2's shape (two 512-thread workgroups per CU, 256 bins) vs pass 1's
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05zf
timeout -k 10 600 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_radix.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zf/tests.log 2>&1 || { echo TESTS FAILED; tail -20 gpurun_out/r05zf/tests.log; exit 1; }
tail -1 gpurun_out/r05zf/tests.log
for k in 1 2; do
  for V in base4 product; do
    if [ $V = product ]; then LIB=$R/mlir-hashjoin_amd/lib/libhj.so; else LIB=$R/build/$V/libhj.so; fi
    HJ_LIB=$LIB timeout -k 10 300 python -u tools/xp_place.py 8 C3 > gpurun_out/r05zf/one.jsonl 2>> gpurun_out/r05zf/err.log || { tail -5 gpurun_out/r05zf/err.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r05zf/one.jsonl'):
    d=json.loads(l); d['variant']='$V'; d['rep']=$k; open('gpurun_out/r05zf/ab.jsonl','a').write(json.dumps(d)+'\n')
"
  done
done
python3 -c "
import json, statistics as st
rows=[json.loads(l) for l in open('gpurun_out/r05zf/ab.jsonl')]
for V in ('base4','product'):
    b=[r['build'] for r in rows if r['variant']==V]; p=[r['probe_partition'] for r in rows if r['variant']==V]
    print(V, 'build mean %.3f max %.3f' % (st.mean(b), max(b)), 'part mean %.3f max %.3f' % (st.mean(p), max(p)), 'draws', rows[-1]['placement'] if V=='product' else '')
"
