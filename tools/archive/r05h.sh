#!/bin/bash
# experiments: contiguous workspaces (per-relation pass spread), workgroup stagger (store phases in step?)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05h; mkdir -p $O; cd $R
M=mlir-hashjoin_amd/micro/bin
for V in "" _stg16 _stg48; do
  timeout -k 10 240 $M/pass_micro$V > $O/pass_micro$V.txt 2>&1 || { echo "pass_micro$V failed"; exit 1; }
done
bash tools/ab_alt.sh r05h "C3" contig 3 || exit 1
bash tools/ab_alt.sh r05h2 "C3" stg16 2 || exit 1
bash tools/ab_alt.sh r05h3 "C3" stg48 2 || exit 1
echo r05h done
