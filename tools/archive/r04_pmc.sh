#!/bin/bash
# round-4: PMC counter sets of bench workloads, each set a --pmc run of its own
#   tools/r04_pmc.sh <tag> "<config[:bench args]> ..." "<counter set>" ["<counter set>" ...]
# e.g. tools/r04_pmc.sh r04l "C3 C3:--force-dist" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum"
set -o pipefail
TAG=$1; SPECS=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for SPEC in $SPECS; do
  C=${SPEC%%:*}; X=""; [ "$SPEC" != "$C" ] && X=${SPEC#*:}
  NAME=$C; [ -n "$X" ] && NAME=$C-dist
  for CNT in "$@"; do
    N=$(echo $CNT | tr ' ' '_' | cut -c1-80)
    timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/${NAME}_$N" -o run -- \
        python3 "$R/bench.py" --config $C $X --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > "$OUT/${NAME}_$N.log" 2>&1 \
        || { rc=$?; echo "pmc $N $NAME failed rc=$rc"; tail -n 3 "$OUT/${NAME}_$N.log"; exit $rc; }
  done
done
echo pmc done
