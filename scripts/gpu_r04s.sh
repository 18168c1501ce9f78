#!/bin/bash
# round 4 final tree: the full GPU suite, smoke, the default bench (with the CPU
# baseline), its rocprof kernel stats, and the C2 / C4 / C5 / reference-layout /
# 2-rank benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
bash scripts/gpu_check.sh r04s tests smoke bench rocprof bench:C2 bench:C4 bench:C5 rank2 || exit $?
O=gpurun_out/r04s
timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout.json" 2> "$O/bench_reflayout.err" || { tail -20 "$O/bench_reflayout.err"; exit 1; }
cut -c1-200 "$O/bench_reflayout.json"
