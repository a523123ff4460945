#!/bin/bash
# round-4: GPU suite, default bench line, then kernel trace + PMC of configs
#   tools/r04_prof.sh <tag> <config>[:args] ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || { echo "default bench failed"; exit 1; }
tail -c 600 gpurun_out/$TAG/bench_default.json
bash profiles/collect_set.sh $TAG "$@"
