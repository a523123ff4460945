#!/bin/bash
# round-4 final (one call): GPU suite, kernel traces + PMC of every bench
# workload, pmc_latest.json from them (here on the box, so the default bench
# line below carries its PMC traffic; regenerated the same way from the
# merged gpurun_out/ at home), every config's bench line, the forced-dist
# line, and bench.py with its defaults.
#   tools/r04_final_all.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -ne 0 ] && exit $rc
bash profiles/collect_set.sh $TAG C3 REF-B C1 C1-ref C4 REF-A C2 C3:--force-dist || exit 1
cd $R
for C in C3 REF-B C1 C1-ref C4 REF-A C2; do
  python3 profiles/pmc_to_json.py gpurun_out/prof_${TAG}_$C $C 1 "profiles/${TAG}_${C}_profile.txt" > /dev/null || exit 1
done
python3 profiles/pmc_to_json.py gpurun_out/prof_${TAG}_C3-dist C3-dist 1 "profiles/${TAG}_C3-dist_profile.txt" > /dev/null || exit 1
for C in C3 C1 C1-ref C2 C4 REF-A REF-B; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
      >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH $C FAILED"; exit 1; }
done
timeout -k 10 300 python -u bench.py --config C3 --force-dist --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 \
    >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "BENCH forced-dist FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err \
    || { echo "DEFAULT BENCH FAILED"; tail -5 gpurun_out/${TAG}_default.err; exit 1; }
cat gpurun_out/${TAG}_default.json | head -c 600
