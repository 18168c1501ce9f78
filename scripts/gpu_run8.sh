#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_fused.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_bench.log 2>&1; rc=$?
cat gpurun_out/conv_bench.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench8.json 2> gpurun_out/bench8.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench8.err | tail -5; cat gpurun_out/bench8.json
exit $rc
