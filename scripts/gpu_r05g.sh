#!/bin/bash
# round 5: the literal drop-in (--reference-api) and the reference-layout path at C3,
# each bench line plus a rocprofv3 --kernel-trace --stats summary
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r05g
mkdir -p $O
for mode in reference-api reference-layout; do
  timeout -k 10 300 python -u bench.py --$mode --no-cpu-baseline > $O/bench_$mode.json 2> $O/bench_$mode.err || { tail -20 $O/bench_$mode.err; exit 1; }
  cat $O/bench_$mode.json
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$mode" -o run --output-format csv -- python3 "$R/bench.py" --$mode --steps 5 --warmup 2 --no-cpu-baseline > "$R/$O/bench_rocprof_$mode.json" 2> "$R/$O/bench_rocprof_$mode.err") || exit 1
  ks=$(find "$O/prof_$mode" -name '*kernel_stats.csv' | head -n 1)
  cp "$ks" "$O/rocprof_kernel_stats_$mode.csv"
  python3 scripts/kstats.py "$O/bench_rocprof_$mode.json" "$O/rocprof_kernel_stats_$mode.csv" > "$O/rocprof_top_$mode.txt"
  head -12 "$O/rocprof_top_$mode.txt"
done
