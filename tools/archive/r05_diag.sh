#!/bin/bash
# Round 5, VERDICT r04 item 1: is the driver's slower S partition a property
# of the box or of a cold start?  On a fresh lease: the driver's exact bench
# command FIRST, then a repeat, then the copy-floor test, a kernel trace and
# PMC passes of the same workload (each counter set a run of its own).
#   tools/r05_diag.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
date +%s > $O/t0
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/first.json 2> $O/first.err \
    || { echo "first bench failed"; tail -5 $O/first.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-leg \
    > $O/second.json 2> $O/second.err || { echo "second bench failed"; exit 1; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_copy.py "tests/test_gpu_radix.py::test_radix_duplicates_across_build_rounds" -x -q --timeout 120 --timeout-method thread \
    > $O/copytest.log 2>&1 || { echo "copy test failed"; tail -20 $O/copytest.log; exit 1; }
tail -1 $O/copytest.log
cd /tmp && export TMPDIR=/tmp
P=$O/prof
mkdir -p $P
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-leg --steps 20 --warmup 5 > $P/trace.log 2>&1 \
    || { echo "trace failed"; tail -5 $P/trace.log; exit 1; }
for CNT in "GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum" FETCH_SIZE WRITE_SIZE; do
  N=$(echo $CNT | tr ' ' '_' | cut -c1-60)
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $P/pmc_$N -o run -- \
      python3 $R/bench.py --no-cpu-baseline --no-host-leg --no-floor --steps 20 --warmup 5 > $P/pmc_$N.log 2>&1 \
      || { rc=$?; echo "pmc $N failed rc=$rc"; tail -3 $P/pmc_$N.log; exit $rc; }
done
echo diag done
