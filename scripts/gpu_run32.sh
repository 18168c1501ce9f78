#!/bin/bash
# ping-pong band conv: parity (band/GRU/dwhead tests), per-conv A/B, chip MFMA peak + shader clock
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 60 scripts/probe/bin/mfma_peak > gpurun_out/mfma_peak.log 2>&1 || exit 1
cat gpurun_out/mfma_peak.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/pytest32.log 2>&1 || { tail -30 gpurun_out/pytest32.log; exit 1; }
tail -3 gpurun_out/pytest32.log
for pp in 0 1; do echo "== PP=$pp"; DROID_CONV_PP=$pp timeout -k 10 120 python scripts/conv_bench.py 2048 2>&1 | grep -v amdgpu || exit 1; done
