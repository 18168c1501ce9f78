#!/bin/bash
# GRU epilogues with preloaded h/z: parity + bench breakdown + kernel stats
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out; R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py > gpurun_out/pytest47.log 2>&1 || { tail -30 gpurun_out/pytest47.log; exit 1; }
tail -2 gpurun_out/pytest47.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof47" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --breakdown --no-cpu-baseline > "$R/gpurun_out/bench47.json" 2> "$R/gpurun_out/bench47.err" || exit 1
cd "$R"; python3 -c "import json; d=json.load(open('gpurun_out/bench47.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'])"
head -8 gpurun_out/prof47/run_kernel_stats.csv | cut -d, -f1-4
