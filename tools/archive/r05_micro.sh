#!/bin/bash
# Round 5: one box, everything that tells a fast pass box from a slow one,
# plus the one-pass micro.
#   tools/r05_micro.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
{ amd-smi static 2>&1 | grep -iE "vram|vendor|type|size|market|product|sku|partition|bus|serial" | head -40
  rocm-smi --showmemvendor --showproductname --showclocks --showmemorypartition --showcomputepartition 2>&1 | head -60
} > $O/box.txt || true
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-leg --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
    || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
M=$R/mlir-hashjoin_amd/micro/bin
timeout -k 10 240 $M/pass_micro > $O/pass_micro.txt 2>&1 || { echo "pass_micro failed"; tail -5 $O/pass_micro.txt; exit 1; }
timeout -k 10 120 $M/frontier_micro > $O/frontier_micro.txt 2>&1 || { echo "frontier_micro failed"; exit 1; }
timeout -k 10 240 $M/onepass_micro > $O/onepass_micro.txt 2>&1 || { echo "onepass_micro failed"; tail -5 $O/onepass_micro.txt; exit 1; }
echo micro done
