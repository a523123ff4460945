#!/bin/bash
# alternating A/B of build/<variant> libraries against the product
#   tools/r06/ab_any.sh <tag> "<configs>" "<variants>" [reps]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash tools/ab_alt.sh "$1" "$2" "$3" ${4:-2}
