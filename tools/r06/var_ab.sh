#!/bin/bash
# a build/<variant> library: parity tests, then alternating A/B against the product
#   tools/r06/var_ab.sh <tag> "<variants>" "<configs>" "<test files>" [reps]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; VS=$2; CS=$3; TS=$4; REPS=${5:-2}
cd $R && mkdir -p gpurun_out/$TAG
for V in $VS; do
  HJ_LIB=$R/build/$V/libhj.so timeout -k 10 600 python -u -m pytest $TS -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests_$V.log 2>&1 || { echo TESTS $V FAILED; tail -30 gpurun_out/$TAG/tests_$V.log; exit 1; }
  echo "$V: $(tail -1 gpurun_out/$TAG/tests_$V.log)"
done
bash tools/ab_alt.sh $TAG "$CS" "$VS" $REPS
