#!/bin/bash
# Band conv kernel: parity tests, then per-conv A/B (band vs row-band kernel).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest_band.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_band.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
DROID_CONV_BAND=0 timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_old.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/conv_old.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_band.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/conv_band.log
exit $rc
