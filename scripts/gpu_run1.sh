#!/bin/bash
# GPU run: tests, smoke, short bench. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
tail -25 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench1.err; cat gpurun_out/bench1.json
exit $rc
