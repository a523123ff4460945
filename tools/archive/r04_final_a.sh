#!/bin/bash
# round-4 final, part A: GPU suite on the product library, then kernel traces
# + PMC of every bench workload (profiles/collect_set.sh)
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
bash profiles/collect_set.sh $TAG C3 REF-B C1 C1-ref C4 REF-A C2 C3:--force-dist
