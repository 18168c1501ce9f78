#!/bin/bash
# fused lookup: two tiles in flight (branch-free buffer gathers, LDS-staged coordinates); tests + bench A/B
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py tests/test_gpu_corr.py > gpurun_out/pytest36.log 2>&1 || { grep -v amdgpu.ids gpurun_out/pytest36.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest36.log
for tv in 0 1; do
  DROID_TILED_VOLUME=$tv timeout -k 10 600 python bench.py --breakdown --no-cpu-baseline > gpurun_out/bench36_$tv.json 2> gpurun_out/bench36_$tv.err || { tail -5 gpurun_out/bench36_$tv.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench36_$tv.json')); print('tiled=$tv', round(d['value'],2), 'it/s', d['breakdown_ms'], d['roofline_lookup']['launch_ms'])"
done
