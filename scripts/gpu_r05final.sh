#!/bin/bash
# round 5, final tree: GPU suite, smoke, the default C3 bench line (CPU baseline
# included, as the driver runs it) and a rocprofv3 --kernel-trace --stats summary of C3
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O="${FINAL_OUT:-gpurun_out/r05final}"
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 1; }
cat $O/bench_C3.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_C3" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/$O/bench_rocprof_C3.json" 2> "$R/$O/bench_rocprof_C3.err") || exit 1
ks=$(find "$O/prof_C3" -name '*kernel_stats.csv' | head -n 1)
cp "$ks" "$O/rocprof_kernel_stats_C3.csv"
python3 scripts/kstats.py "$O/bench_rocprof_C3.json" "$O/rocprof_kernel_stats_C3.csv" > "$O/rocprof_top_C3.txt"
head -14 "$O/rocprof_top_C3.txt"
