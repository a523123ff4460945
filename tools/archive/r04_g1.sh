set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04a
timeout -k 10 120 ./mlir-hashjoin_amd/micro/bin/direct_micro > gpurun_out/r04a/direct_micro.txt 2>&1
echo micro rc $?
timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 > gpurun_out/r04a/c3.json 2> gpurun_out/r04a/c3.err && echo bench ok
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04a/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --no-host-leg --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r04a/trace.log 2>&1 && echo trace ok
