#!/bin/bash
# Round 6: the per-wave output claims (k_join_b) -- GPU suite, then an
# alternating A/B against the round-5 scan path (build/old: HJ_WAVE_CLAIM=0)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06b}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1 || { tail -40 gpurun_out/$TAG/gputest.log; exit 1; }
tail -1 gpurun_out/$TAG/gputest.log
bash tools/ab_alt.sh $TAG "${2:-C3 REF-B C1-ref C4 C1}" old ${3:-2}
