#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01b" -o bench --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench7.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench7.err"
rc=$?; echo "rc=$rc"; cat "$GRAFT_REPO_ROOT/gpurun_out/bench7.json"; exit $rc
