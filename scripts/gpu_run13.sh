#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -5 gpurun_out/pmc_traffic.log
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/profiles_new && cp profiles/pmc_*.json gpurun_out/profiles_new/
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench13.json 2> gpurun_out/bench13.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench13.err | tail -5; cat gpurun_out/bench13.json
exit $rc
