#!/bin/bash
# Round 6: per-wave output claims, nt vs plain ballot stores, against build/old
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06d}
cd $R && mkdir -p gpurun_out/$TAG
bash tools/ab_alt.sh $TAG "${2:-C3 REF-B}" "old plain" ${3:-2} || exit 1
