#!/bin/bash
# round-4: GPU suite on the product library, then A/B bench lines of experiment builds
#   tools/r04_ab.sh <tag> "<configs>" <variant> ...
set -o pipefail
TAG=$1; CONFIGS=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $TAG "$CONFIGS" "$@"
