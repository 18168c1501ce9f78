#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py -k "dw_head or update" > gpurun_out/pytest48.log 2>&1 || { tail -30 gpurun_out/pytest48.log; exit 1; }
tail -2 gpurun_out/pytest48.log
for c in dwh; do timeout -k 10 120 python scripts/conv_timeline.py 2048 $c 2>&1 | grep -v amdgpu || exit 1; done
timeout -k 10 120 python scripts/conv_bench.py 2048 dwhead 2>&1 | grep -v amdgpu
