#!/bin/bash
# round 6: Cholesky rework - BA tests, timeline, same-box BA A/B, C3 bench + rocprof (no CPU baseline)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py tests/test_gpu_trajectory.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || exit 1
grep -E "span|potrf tasks|panels \(|second|back solve" $O/chol_timeline_C3.txt
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_new_$rep.txt 2>&1 || exit 1
  DROID_HIP_LIB=droid-slam_amd/lib/prev/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prev_$rep.txt 2>&1 || exit 1
done
grep -h "ba(itrs" $O/ba_*.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 1; }
cat $O/bench_C3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_C3" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/$O/bench_rocprof_C3.json" 2> "$R/$O/bench_rocprof_C3.err") || exit 1
ks=$(find "$O/prof_C3" -name '*kernel_stats.csv' | head -n 1)
cp "$ks" "$O/rocprof_kernel_stats_C3.csv"
python3 scripts/kstats.py "$O/bench_rocprof_C3.json" "$O/rocprof_kernel_stats_C3.csv" > "$O/rocprof_top_C3.txt"
head -16 "$O/rocprof_top_C3.txt"
