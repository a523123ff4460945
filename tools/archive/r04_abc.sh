#!/bin/bash
# round-4: GPU suite on the product library and on each CHECK variant
# (HJ_LIB=build/<v>/libhj.so), then A/B bench lines of the variants
#   tools/r04_abc.sh <tag> "<configs>" "<check variants>" <variant> ...
set -o pipefail
TAG=$1; CONFIGS=$2; CHECK=$3; shift 3
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
for V in $CHECK; do
  HJ_LIB=$R/build/$V/libhj.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/$TAG/gputest_$V.log 2>&1; rc=$?
  echo "check $V:"; tail -2 gpurun_out/$TAG/gputest_$V.log
  [ $rc -ne 0 ] && exit $rc
done
bash tools/ab_libs.sh $TAG "$CONFIGS" "$@"
