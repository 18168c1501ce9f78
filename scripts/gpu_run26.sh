#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_fused.py -q -rf -x -k "alt or pyramid or lookup_ce0" > gpurun_out/pytest26.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest26.log | tail -30; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline --corr pyramid > gpurun_out/bench26.json 2> gpurun_out/bench26.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench26.json; grep -v amdgpu gpurun_out/bench26.err | tail -5; exit $rc
