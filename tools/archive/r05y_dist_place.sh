#!/bin/bash
# routed-tuple buffers placement-probed: dist GPU tests, forced-dist C3 off / on / off / on, kernel trace (on)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05y
timeout -k 10 900 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_dist.py tests/test_gpu_radix.py tests/test_gpu_parity.py tests/test_gpu_skew.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05y/tests.log; exit 1; }
tail -1 gpurun_out/r05y/tests.log
for k in 1 2; do
  for P in 0 1; do
    HJ_PLACEMENT_PROBE=$P timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
        > gpurun_out/r05y/one.json 2>> gpurun_out/r05y/bench.err || { echo "bench failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05y/one.json')); d['probe_env']='$P'; open('gpurun_out/r05y/ab.jsonl','a').write(json.dumps(d)+'\n'); print('$P', d['ms_per_step'], {k:round(v,3) for k,v in d['phase_ms'].items() if v}, d['placement'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05y/trace_dist -o run -- \
    python3 $R/bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $R/gpurun_out/r05y/trace_dist.log 2>&1 || echo "trace rc=$?"
cd $R
for C in REF-B C1-ref; do
  HJ_PLACEMENT_PROBE=0 timeout -k 10 200 python -u tools/xp_place.py 8 $C > gpurun_out/r05y/${C}_place_off.jsonl 2>> gpurun_out/r05y/bench.err || echo "$C off failed"
  timeout -k 10 200 python -u tools/xp_place.py 8 $C > gpurun_out/r05y/${C}_place_on.jsonl 2>> gpurun_out/r05y/bench.err || echo "$C on failed"
done
bash tools/ab_alt.sh r05y_dbl "C3 C4 C1" base2 2
HJ_LIB=$R/build/wdyn/libhj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_skew.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y/tests_wdyn.log 2>&1 || { echo WDYN TESTS FAILED; tail -20 gpurun_out/r05y/tests_wdyn.log; exit 1; }
tail -1 gpurun_out/r05y/tests_wdyn.log
bash tools/ab_alt.sh r05y_wdyn "C3 C4" wdyn 2
