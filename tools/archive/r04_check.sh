#!/bin/bash
# round-4 GPU check: optional micros, then the GPU suite.
#   tools/r04_check.sh <tag> [micro ...]
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
for m in "$@"; do
  timeout -k 10 300 ./mlir-hashjoin_amd/micro/bin/$m > gpurun_out/$TAG/$m.txt 2>&1 || { echo "$m FAILED rc=$?"; exit 1; }
  echo "$m ok"
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
exit $rc
