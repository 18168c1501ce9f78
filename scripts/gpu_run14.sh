#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_chol.py -q -rf -x > gpurun_out/pytest_chol.log 2>&1; rc=$?
echo "chol rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_chol.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_ba.py tests/test_gpu_update.py -q -rf -x > gpurun_out/pytest_ba.log 2>&1; rc=$?
echo "ba rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_ba.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/ba_bench.py C3 5 > gpurun_out/ba_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ba_bench.log | tail -8
DROID_CHOL=blocked timeout -k 10 300 python scripts/ba_bench.py C3 5 > gpurun_out/ba_bench_blocked.log 2>&1
grep -v amdgpu.ids gpurun_out/ba_bench_blocked.log | tail -8
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench14.json 2> gpurun_out/bench14.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench14.err | tail -5; cat gpurun_out/bench14.json
exit $rc
