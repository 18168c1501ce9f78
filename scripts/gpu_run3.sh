#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_corr.py -q -rf > gpurun_out/pytest_corr.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_corr.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python scripts/conv_ab.py 2048 > gpurun_out/conv_ab.log 2>&1; rc=$?
echo "conv_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_ab.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01" -o bench --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench3.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench3.err"
rc=$?
echo "rocprof bench rc=$rc"; cat "$GRAFT_REPO_ROOT/gpurun_out/bench3.json"; find "$GRAFT_REPO_ROOT/gpurun_out/prof_r01" -name "*stats*"
exit $rc
