#!/bin/bash
# factored-gate epilogue experiment: pre map L2-resident (all edges -> frame 0) vs 8 edges per frame
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
for k in zrp qp; do
  timeout -k 10 120 python -u scripts/conv_timeline.py 2048 $k > gpurun_out/tl53_$k.txt 2>&1 || { cat gpurun_out/tl53_$k.txt; exit 1; }; cat gpurun_out/tl53_$k.txt
  TL_PIDX0=1 timeout -k 10 120 python -u scripts/conv_timeline.py 2048 $k > gpurun_out/tl53_${k}_0.txt 2>&1 || { cat gpurun_out/tl53_${k}_0.txt; exit 1; }; cat gpurun_out/tl53_${k}_0.txt
done
