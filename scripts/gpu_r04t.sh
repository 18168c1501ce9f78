#!/bin/bash
# round 4: kernel breakdowns of C5 and C2 (rocprof stats), and C3 with the
# on-demand lookup (no volume) for the volume-free comparison
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
bash scripts/gpu_check.sh r04t rocprof:C5 rocprof:C2 || exit $?
O=gpurun_out/r04t
timeout -k 10 600 python -u bench.py --corr pyramid --no-cpu-baseline > "$O/bench_C3_pyramid.json" 2> "$O/bench_C3_pyramid.err" || { tail -20 "$O/bench_C3_pyramid.err"; exit 1; }
cut -c1-300 "$O/bench_C3_pyramid.json"
