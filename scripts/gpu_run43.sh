#!/bin/bash
# compile-time epilogue type in the band conv: parity, per-conv timing, timeline
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py > gpurun_out/pytest43.log 2>&1 || { tail -30 gpurun_out/pytest43.log; exit 1; }
tail -2 gpurun_out/pytest43.log
timeout -k 10 120 python scripts/conv_bench.py 2048 2>&1 | grep -v amdgpu || exit 1
for c in q ce2; do timeout -k 10 120 python scripts/conv_timeline.py 2048 $c 2>&1 | grep -v amdgpu || exit 1; done
