#!/bin/bash
# round-4 GPU check: the GPU suite, then bench lines, then a C3 kernel trace.
#   tools/r04_full.sh <tag> [config ...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
for C in "$@"; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/$TAG/bench.jsonl 2>> gpurun_out/$TAG/bench.err || { echo "BENCH $C FAILED"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- \
    python3 $R/bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $R/gpurun_out/$TAG/trace.log 2>&1
echo "trace rc $?"
