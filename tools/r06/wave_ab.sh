#!/bin/bash
# Round 6: A/B of the per-wave output claims against build/old, then a
# kernel trace of the product on C3 (k_join_b alone, k_out_fixup)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06c}
cd $R && mkdir -p gpurun_out/$TAG
bash tools/ab_alt.sh $TAG "${2:-C3 REF-B}" old ${3:-2} || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --config ${4:-C3} --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $R/gpurun_out/$TAG/prof.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/prof.log; exit 1; }
f=$(find $R/gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -14
