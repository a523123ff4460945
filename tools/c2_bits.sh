cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 9 8 10; do
  timeout -k 10 200 python -u bench.py --config C2 --radix-bits $b --no-cpu-baseline --no-host-leg --steps 10 --warmup 3 > gpurun_out/c2b$b.json 2>gpurun_out/c2b$b.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c2b$b.json')); print($b, d['ms_per_step'], d['phase_ms'], d['roofline']['kernel']['name'][:20])"
done
