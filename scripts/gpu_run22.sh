#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof22" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/bench22_prof.json" 2> "$R/gpurun_out/bench22_prof.err"; rc=$?
echo "prof rc=$rc"; exit $rc
