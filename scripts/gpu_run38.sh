#!/bin/bash
# fused lookup with packed-fp16 bilinear arithmetic: bit-exact tests, bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py tests/test_gpu_corr.py > gpurun_out/pytest38.log 2>&1 || { grep -v amdgpu.ids gpurun_out/pytest38.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest38.log
timeout -k 10 600 python bench.py --breakdown --no-cpu-baseline > gpurun_out/bench38.json 2> gpurun_out/bench38.err || { tail -5 gpurun_out/bench38.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench38.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'], d['roofline_lookup'])"
