#!/bin/bash
# round-4: write-request counters of the partition passes (EXACT routing pass
# vs the bucketed passes), C3 and C3 --force-dist, each counter set a --pmc
# run of its own; plus the forced-dist bench line.
#   tools/r04_wr.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || echo "list failed"
timeout -k 10 300 python3 $R/bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    > $OUT/bench_dist.json 2> $OUT/bench_dist.err || { echo "bench dist failed"; exit 1; }
for SPEC in C3 C3:--force-dist; do
  C=${SPEC%%:*}; X=""; [ "$SPEC" != "$C" ] && X=${SPEC#*:}
  NAME=$C; [ -n "$X" ] && NAME=$C-dist
  for CNT in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCP_TCC_WRITE_REQ_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    N=$(echo $CNT | tr ' ' '_')
    timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/${NAME}_$N" -o run -- \
        python3 "$R/bench.py" --config $C $X --no-cpu-baseline --no-host-leg --steps 3 --warmup 1 > "$OUT/${NAME}_$N.log" 2>&1 \
        || { rc=$?; echo "pmc $N $NAME failed rc=$rc"; tail -3 "$OUT/${NAME}_$N.log";
             [ $rc -ge 124 ] && exit $rc; }
  done
done
echo all done
