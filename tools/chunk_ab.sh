#!/bin/bash
# (Runs against the library of commit b41946e: the HJ_CHUNKS code was removed after the measurement, profiles/r03_chunked_handoff.txt.)
# A/B of the chunked probe (HJ_CHUNKS, HJ_CHUNK_STREAMS): C3 bench lines with verification, then a kernel trace.
set -e
mkdir -p gpurun_out/chunk
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-leg --verify \
    > gpurun_out/chunk/c3_$name.json 2> gpurun_out/chunk/c3_$name.err
  python -c "import json; d=json.load(open('gpurun_out/chunk/c3_$name.json')); print('$name', d['ms_per_step'], d['phase_ms'])"
}
run k0 HJ_CHUNKS=0
for k in 4 8 16 32 64; do run s2k$k HJ_CHUNKS=$k HJ_CHUNK_STREAMS=2; done
K=${TRACE_K:-16}
HJ_CHUNKS=$K HJ_CHUNK_STREAMS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chunk/trace2 -o c3 -- python -u bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-leg > gpurun_out/chunk/trace2.log 2>&1
