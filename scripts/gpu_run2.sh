#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python tests/debug_corr16.py > gpurun_out/debug16.log 2>&1; rc=$?
echo "debug rc=$rc"; cat gpurun_out/debug16.log | grep -v amdgpu.ids
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench2.err | tail -8; cat gpurun_out/bench2.json
exit $rc
