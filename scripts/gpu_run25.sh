#!/bin/bash
# Full round check: GPU parity suite, smoke, default bench (with cpu_baseline), rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_e.err | tail -5; cat gpurun_out/bench_e.json
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --breakdown --no-cpu-baseline > gpurun_out/bench_e_prof.json 2> gpurun_out/bench_e_prof.err; rc=$?
echo "prof rc=$rc"; cat gpurun_out/bench_e_prof.json
exit $rc
