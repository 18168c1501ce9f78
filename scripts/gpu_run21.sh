#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_fused.py tests/test_gpu_update.py -q -rf -x > gpurun_out/pytest21.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest21.log | tail -25; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline > gpurun_out/bench21.json 2> gpurun_out/bench21.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench21.json; if [ $rc -ne 0 ]; then tail gpurun_out/bench21.err; exit $rc; fi
