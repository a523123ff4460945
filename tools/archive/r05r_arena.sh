#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r05r
HJ_LIB=build/xppad/libhj.so timeout -k 10 300 python -u tools/xp_pad.py arena > gpurun_out/r05r/arena.jsonl 2> gpurun_out/r05r/arena.err || { tail -5 gpurun_out/r05r/arena.err; exit 1; }
cat gpurun_out/r05r/arena.jsonl
cd /tmp && export TMPDIR=/tmp
HJ_LIB=$R/build/xppad/libhj.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05r/trace -o run -- python3 $R/tools/xp_pad.py arena > $R/gpurun_out/r05r/trace.log 2>&1 || { echo trace failed; tail -5 $R/gpurun_out/r05r/trace.log; exit 1; }
