#!/bin/bash
# gru_glo: 5-tile ring (4 in flight): parity + bench + stats
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out; R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py > gpurun_out/pytest67.log 2>&1 || { tail -40 gpurun_out/pytest67.log; exit 1; }
tail -1 gpurun_out/pytest67.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof67" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/bench67.json" 2> "$R/gpurun_out/bench67.err" || exit 1
cd "$R"; python3 scripts/kstats.py gpurun_out/bench67.json gpurun_out/prof67/run_kernel_stats.csv segment glo flow_enc0
