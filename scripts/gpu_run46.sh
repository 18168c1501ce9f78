#!/bin/bash
# Full round check after the dataflow-Cholesky rewrite: GPU parity suite, smoke, default bench
# (with cpu_baseline), rocprofv3 kernel stats; GRBM clock counters around the ZR conv.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; R=$(pwd)
mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu46.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu46.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke46.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke46.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench46.json 2> gpurun_out/bench46.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench46.json
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof46" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --breakdown --no-cpu-baseline > "$R/gpurun_out/bench46_prof.json" 2> "$R/gpurun_out/bench46_prof.err"; rc=$?
echo "prof rc=$rc"; cat "$R/gpurun_out/bench46_prof.json"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/pmc_clk46" -o c --output-format csv -- python3 "$R/scripts/conv_bench.py" 2048 zr > "$R/gpurun_out/pmc_clk46.log" 2>&1; rc=$?
echo "pmc rc=$rc"; grep -v amdgpu "$R/gpurun_out/pmc_clk46.log" | grep "zr"
exit $rc
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_traffic46/$c" -o w --output-format csv -- python3 "$R/scripts/pmc_workload.py" > "$R/gpurun_out/pmc_traffic46_$c.log" 2>&1 || exit 1
done
echo "traffic passes ok"
