#!/bin/bash
# per-rank cost at N=8 strong scaling ~ the same graph with 1/8 of the edges on one GPU
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for e in 2048 512 256; do
  timeout -k 10 600 python bench.py --edges $e --breakdown --no-cpu-baseline > gpurun_out/bench40_$e.json 2> gpurun_out/bench40_$e.err || { tail -5 gpurun_out/bench40_$e.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench40_$e.json')); print('edges=$e', round(d['value'],2), 'it/s', round(d['ms_per_step'],2), 'ms', {k: round(v,3) for k,v in d['breakdown_ms'].items()})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof40" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --edges 256 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
head -25 "$GRAFT_REPO_ROOT/gpurun_out/prof40/run_kernel_stats.csv" | cut -c1-160
