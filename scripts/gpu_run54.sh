#!/bin/bash
# band epilogue sub-phase timeline (profiling build), z|r and q with / without the per-frame term
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
for k in zr zrp q qp; do
  timeout -k 10 120 python -u scripts/conv_timeline.py 2048 $k > gpurun_out/tl54_$k.txt 2>&1 || { cat gpurun_out/tl54_$k.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/tl54_$k.txt
done
