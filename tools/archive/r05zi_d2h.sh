#!/bin/bash
# host-memref outputs through page-locked staging: host-path tests, then the bench's host leg A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05zi
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c_driver.py tests/test_gpu_rows.py tests/test_gpu_ooc.py tests/test_gpu_select.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zi/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05zi/tests.log; exit 1; }
tail -1 gpurun_out/r05zi/tests.log
for k in 1 2; do
  for V in base6 product; do
    if [ $V = product ]; then LIB=$R/mlir-hashjoin_amd/lib/libhj.so; else LIB=$R/build/$V/libhj.so; fi
    HJ_LIB=$LIB timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline --no-floor --steps 3 --warmup 1 > gpurun_out/r05zi/one.json 2>> gpurun_out/r05zi/err.log || { tail -5 gpurun_out/r05zi/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r05zi/one.json')); h=d['host_memref']; h['variant']='$V'; h['rep']=$k
open('gpurun_out/r05zi/ab.jsonl','a').write(json.dumps(h)+'\n'); print('$V', h['count_ms'], h['probe_ms'], h['download_ms'], h['probe_tuples_per_s_end_to_end'])"
  done
done
