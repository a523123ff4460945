#!/bin/bash
# (Runs against the library of commit b41946e: the HJ_CHUNKS code was removed after the measurement, profiles/r03_chunked_handoff.txt.)
# Does S's pass-2 -> join hand-off come from the Infinity Cache?  Chunked probe (HJ_CHUNKS=K) with each
# chunk's join right after its pass ("inter") against every pass first, then every join ("split": the
# same launches and tails, no hand-off).  Kernel traces of each; summarised by tools/chunk_summary.py.
set -e
mkdir -p gpurun_out/handoff
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in 16 32 64; do
  for mode in inter split; do
    if [ $mode = split ]; then export HJ_CHUNK_SPLIT=1; else unset HJ_CHUNK_SPLIT; fi
    HJ_CHUNKS=$k timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/handoff/k${k}_$mode -o t -- \
      python -u bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-leg \
      > gpurun_out/handoff/k${k}_$mode.json 2> gpurun_out/handoff/k${k}_$mode.err
    echo "k=$k $mode done"
  done
done
unset HJ_CHUNK_SPLIT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/handoff/k0 -o t -- \
  python -u bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-leg > gpurun_out/handoff/k0.json 2> gpurun_out/handoff/k0.err
