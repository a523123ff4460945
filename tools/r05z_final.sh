#!/bin/bash
# GPU suite + the driver's bench command, then trace + PMC of the given configs
#   tools/r05z_final.sh <tag> <config>...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
bash $R/tools/r05_check.sh $TAG || exit 1
bash $R/profiles/collect_set.sh $TAG "$@" || exit 1
