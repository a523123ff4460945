#!/bin/bash
# Round 6: per-wave k_join_b item phases of experiment builds (HJ_XP_PHASES)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06f}; shift
cd $R && mkdir -p gpurun_out/$TAG
for C in ${CONFIGS:-C3 REF-B}; do
  for V in "$@"; do
    HJ_LIB=$R/build/$V/libhj.so timeout -k 10 300 python -u tools/r06/xp_phases.py $C >> gpurun_out/$TAG/phases.txt 2>&1 || { tail -20 gpurun_out/$TAG/phases.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/$TAG/phases.txt
