#!/bin/bash
# round 5 final tree: rocprofv3 --kernel-trace --stats of the C5 bench (per-update breakdown)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r05c5
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_C5" -o run --output-format csv -- python3 "$R/bench.py" --config C5 --steps 2 --warmup 1 --no-cpu-baseline > "$R/$O/bench_rocprof_C5.json" 2> "$R/$O/bench_rocprof_C5.err") || exit 1
ks=$(find "$O/prof_C5" -name '*kernel_stats.csv' | head -n 1)
cp "$ks" "$O/rocprof_kernel_stats_C5.csv"
python3 scripts/kstats.py "$O/bench_rocprof_C5.json" "$O/rocprof_kernel_stats_C5.csv" > "$O/rocprof_top_C5.txt"
head -16 "$O/rocprof_top_C5.txt"
