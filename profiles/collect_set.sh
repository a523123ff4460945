#!/bin/bash
# rocprofv3 kernel trace + PMC (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) of
# several bench workloads, each pass in its own run (MI355X_MICROARCH.md:
# never --pmc together with trace domains).
#   profiles/collect_set.sh <tag> <config>[:extra-bench-args] ...
# e.g. profiles/collect_set.sh r03a C3 C1-ref C3:--force-dist
# Output: gpurun_out/prof_<tag>_<config>[-dist]/{trace,pmc_*}/
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for SPEC in "$@"; do
  C=${SPEC%%:*}; X=""; [ "$SPEC" != "$C" ] && X=${SPEC#*:}
  NAME=$C; [[ "$X" == *--force-dist* ]] && NAME=$C-dist
  OUT=$R/gpurun_out/prof_${TAG}_$NAME
  mkdir -p "$OUT"
  echo "== $NAME" 
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 "$R/bench.py" --config $C $X --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > "$OUT/trace.log" 2>&1 \
      || { echo "trace $NAME failed"; tail -5 "$OUT/trace.log"; exit 1; }
  for CNT in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    N=$(echo $CNT | tr ' ' '_')
    timeout -k 10 240 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/pmc_$N" -o run -- \
        python3 "$R/bench.py" --config $C $X --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > "$OUT/pmc_$N.log" 2>&1 \
        || { echo "pmc $N $NAME failed"; tail -5 "$OUT/pmc_$N.log"; exit 1; }
  done
  echo done > "$OUT/DONE"
done
