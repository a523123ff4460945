#!/bin/bash
# pass_micro on the fixed pass kernel; forced-distributed C3 with a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05e; mkdir -p $O; cd $R
timeout -k 10 240 mlir-hashjoin_amd/micro/bin/pass_micro > $O/pass_micro.txt 2>&1 || { echo pass_micro failed; tail -5 $O/pass_micro.txt; exit 1; }
timeout -k 10 300 python3 bench.py --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 > $O/dist.json 2> $O/dist.err || { echo dist bench failed; tail -5 $O/dist.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_dist -o run -- \
    python3 $R/bench.py --force-dist --no-cpu-baseline --no-host-leg --no-floor --steps 5 --warmup 2 > $O/trace_dist.log 2>&1 || { echo trace failed; exit 1; }
echo r05e done
