#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?
echo "pytest(halo8) rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_fused.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
DROID_CONV_HALO=4 timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -rf -x -k conv > gpurun_out/pytest_fused4.log 2>&1; rc=$?
echo "pytest(halo4) rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_fused4.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0 4 8; do
  echo "== DROID_CONV_HALO=$v"
  DROID_CONV_HALO=$v timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_bench$v.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/conv_bench$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench9.json 2> gpurun_out/bench9.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench9.err | tail -5; cat gpurun_out/bench9.json
exit $rc
