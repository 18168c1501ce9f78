#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/ba_bench.py C3 5 2>&1 | grep -v amdgpu.ids; rc=$?
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ba" -o ba --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/ba_bench.py" C3 3 2>&1 | grep -v amdgpu.ids | tail -3
