#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
M=$R/mlir-hashjoin_amd/micro/bin/place_micro
cd $R && mkdir -p gpurun_out/r05u
timeout -k 10 100 $M 12 -1 1 > gpurun_out/r05u/plain.txt 2>&1 || { cat gpurun_out/r05u/plain.txt; exit 1; }
timeout -k 10 100 $M 12 4 1 > gpurun_out/r05u/contig.txt 2>&1 || { cat gpurun_out/r05u/contig.txt; exit 1; }
cat gpurun_out/r05u/plain.txt gpurun_out/r05u/contig.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/gpurun_out/r05u/pmc -o run -- $M 12 -1 1 > $R/gpurun_out/r05u/pmc.log 2>&1 || echo "pmc rc=$?"
