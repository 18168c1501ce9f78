#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --breakdown > gpurun_out/bench4.json 2> gpurun_out/bench4.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench4.err | tail -5; cat gpurun_out/bench4.json
exit $rc
