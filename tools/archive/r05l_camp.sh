#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05l
for PRE in 0 1000 3000 7000 0 333; do
  timeout -k 10 60 mlir-hashjoin_amd/micro/bin/camp_micro $PRE >> gpurun_out/r05l/camp.txt 2>&1 || { echo "camp $PRE failed"; exit 1; }
done
cat gpurun_out/r05l/camp.txt
