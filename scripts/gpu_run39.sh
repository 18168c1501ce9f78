#!/bin/bash
# band conv: interleaved fragment reads (ILV) vs compiler schedule - parity + per-conv A/B
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/pytest39.log 2>&1 || { tail -30 gpurun_out/pytest39.log; exit 1; }
tail -2 gpurun_out/pytest39.log
for ilv in 0 1 0 1; do echo "== ILV=$ilv"; DROID_CONV_ILV=$ilv timeout -k 10 120 python scripts/conv_bench.py 2048 2>&1 | grep -v amdgpu || exit 1; done
