#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest23.log 2>&1; rc=$?
echo "pytest(ring) rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest23.log | tail -15; if [ $rc -ne 0 ]; then exit $rc; fi
DROID_CONV_RING=0 timeout -k 10 300 python -m pytest tests/test_gpu_fused.py -q -rf -x > gpurun_out/pytest23b.log 2>&1; rc=$?
echo "pytest(band) rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest23b.log | tail -3; if [ $rc -ne 0 ]; then exit $rc; fi
DROID_CONV_RING=0 timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_old.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/conv_old.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/conv_bench.py 2048 > gpurun_out/conv_ring.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/conv_ring.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline > gpurun_out/bench23.json 2> gpurun_out/bench23.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench23.json; exit $rc
