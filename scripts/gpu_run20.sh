#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/conv_bench.py 2048 dwhead > gpurun_out/conv_dwhead.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/conv_dwhead.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline > gpurun_out/bench20.json 2> gpurun_out/bench20.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench20.json; if [ $rc -ne 0 ]; then tail gpurun_out/bench20.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof20" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/bench20_prof.json" 2> "$R/gpurun_out/bench20_prof.err"; rc=$?
echo "prof rc=$rc"; exit $rc
