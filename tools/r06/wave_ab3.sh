#!/bin/bash
# Round 6: per-wave output claims -- per-wave item phases (xpn: wave claims,
# xpo: the round-5 scan), then nt vs plain stores against build/old
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06e}
cd $R && mkdir -p gpurun_out/$TAG
for C in C3 REF-B; do
  for V in xpo xpn; do
    HJ_LIB=$R/build/$V/libhj.so timeout -k 10 300 python -u tools/r06/xp_phases.py $C >> gpurun_out/$TAG/phases.txt 2>&1 || { tail -20 gpurun_out/$TAG/phases.txt; exit 1; }
  done
done
cat gpurun_out/$TAG/phases.txt
bash tools/ab_alt.sh $TAG "${2:-C3 REF-B}" "old plain" ${3:-2} || exit 1
