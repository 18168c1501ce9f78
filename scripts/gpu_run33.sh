#!/bin/bash
# pipelined band loop: parity of the band/GRU/dwhead convs, then per-conv A/B (PIPE x BAND)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/pytest33.log 2>&1 || { tail -30 gpurun_out/pytest33.log; exit 1; }
tail -3 gpurun_out/pytest33.log
for cfg in "0 1" "1 1" "1 2" "0 2"; do set -- $cfg
  echo "== PIPE=$1 BAND=$2"
  DROID_CONV_PIPE=$1 DROID_CONV_BAND=$2 timeout -k 10 120 python scripts/conv_bench.py 2048 2>&1 | grep -v amdgpu || exit 1
done
