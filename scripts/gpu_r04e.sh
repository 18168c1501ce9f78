#!/bin/bash
# round 4: C3 bench (fused path) and the reference-layout drop-in bench (new / round-3 lookup kernel)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04e"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --breakdown > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout.json" 2> "$O/bench_reflayout.err" || { tail -20 "$O/bench_reflayout.err"; exit 1; }
cat "$O/bench_reflayout.json"
DROID_LOOKUP_V1=1 timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout_v1.json" 2> "$O/bench_reflayout_v1.err" || { tail -20 "$O/bench_reflayout_v1.err"; exit 1; }
cat "$O/bench_reflayout_v1.json"
