#!/bin/bash
# round-4 experiment: kernel trace of C3 --force-dist with the EXACT pass
# writing workgroup-major slots (build/wgm; the join's results are not
# checked by this run -- the pass's time is what is measured)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04q
cd /tmp && export TMPDIR=/tmp
for V in product wgm; do
  if [ $V = product ]; then LIB=$R/mlir-hashjoin_amd/lib/libhj.so; else LIB=$R/build/$V/libhj.so; fi
  HJ_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04q/$V -o run -- \
      python3 $R/bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 \
      > $R/gpurun_out/r04q/$V.log 2>&1; rc=$?
  echo "$V rc=$rc"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
