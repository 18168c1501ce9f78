#!/bin/bash
# q with the per-frame term loaded before pass 1: parity, timelines, bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py tests/test_gpu_corr.py > gpurun_out/pytest59.log 2>&1 || { tail -40 gpurun_out/pytest59.log; exit 1; }
tail -2 gpurun_out/pytest59.log
for k in zrp qp; do
  timeout -k 10 120 python -u scripts/conv_timeline.py 2048 $k > gpurun_out/tl59_$k.txt 2>&1 || { cat gpurun_out/tl59_$k.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/tl59_$k.txt
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --breakdown > gpurun_out/bench59.json 2> gpurun_out/bench59.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench59.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'])"
