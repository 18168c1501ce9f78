#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_fused.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "0 t1" "4 t1" "8 t1" "4 t0" "4 t3"; do
  set -- $v
  lib=""
  if [ "$2" != "t1" ]; then lib="$PWD/droid-slam_amd/lib/variants/libdroid_hip_$2.so"; fi
  echo "== halo $1 issue $2"
  DROID_HIP_LIB=$lib DROID_CONV_HALO=$1 timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/cb.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/cb.log | cat
  if [ $rc -ne 0 ]; then exit $rc; fi
done
