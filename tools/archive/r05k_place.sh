#!/bin/bash
# Pass speed vs process order and workspace allocation flags (hipExtMallocWithFlags
# hipDeviceMallocContiguous = 4 via the HJ_MALLOC_FLAGS experiment knob).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05k
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      > gpurun_out/r05k/one.json 2>> gpurun_out/r05k/err.log || { echo "bench $tag failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05k/one.json')); p=d['phase_ms']; d['variant']='$tag'; open('gpurun_out/r05k/runs.jsonl','a').write(json.dumps(d)+'\n'); print('$tag', d['ms_per_step'], 'build', p['build'], 'part', p['probe_partition'], 'join', p['probe_join'])"
}
run plain1 && run plain2 && run plain3 && run contig1 HJ_MALLOC_FLAGS=4 && run contig2 HJ_MALLOC_FLAGS=4 && run contig3 HJ_MALLOC_FLAGS=4 \
  && run plain4 && run plain5 && run contig4 HJ_MALLOC_FLAGS=4 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/r05k/avail.txt 2>&1 || echo "list-avail rc=$?"
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r05k/pmc_utcl1 -o run -- \
    python3 $R/bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $R/gpurun_out/r05k/pmc_utcl1.log 2>&1 || echo "pmc rc=$?"
