#!/bin/bash
# SQ (wave-state / LDS) counters for one bench workload, two PMC passes of
# their own (MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ per pass).
#   profiles/collect_sq.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES --output-format csv -d "$OUT/a" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 "$@" > "$OUT/a.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM \
    SQ_INST_LEVEL_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/b" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 "$@" > "$OUT/b.log" 2>&1
echo done > "$OUT/DONE"
