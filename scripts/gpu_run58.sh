#!/bin/bash
# operand-swapped 384-row band tiles (8-B epilogue staging writes), LDS-staged biases: parity, timelines, bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py tests/test_gpu_corr.py > gpurun_out/pytest58.log 2>&1 || { tail -40 gpurun_out/pytest58.log; exit 1; }
tail -2 gpurun_out/pytest58.log
for k in zrp qp ce2 dwh; do
  timeout -k 10 120 python -u scripts/conv_timeline.py 2048 $k > gpurun_out/tl58_$k.txt 2>&1 || { cat gpurun_out/tl58_$k.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/tl58_$k.txt
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --breakdown > gpurun_out/bench58.json 2> gpurun_out/bench58.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench58.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'])"
