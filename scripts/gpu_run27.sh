#!/bin/bash
# Re-entry check: GPU parity suite, smoke, default bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu27.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu27.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke27.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke27.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --breakdown --no-cpu-baseline > gpurun_out/bench27.json 2> gpurun_out/bench27.err; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench27.err | tail -25; cat gpurun_out/bench27.json
exit $rc
