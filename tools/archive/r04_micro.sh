#!/bin/bash
# round-4 micro runs on the GPU box: tools/r04_micro.sh <tag> <micro> [<micro> ...]
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
for m in "$@"; do
  timeout -k 10 300 ./mlir-hashjoin_amd/micro/bin/$m > gpurun_out/$TAG/$m.txt 2>&1 || { echo "$m FAILED rc=$?"; exit 1; }
  echo "$m ok"
done
