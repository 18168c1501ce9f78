#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py tests/test_gpu_ba.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_fused.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/ba_bench.py C3 5 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python scripts/chol_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench6.json 2> gpurun_out/bench6.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench6.err | tail -5; cat gpurun_out/bench6.json
exit $rc
