#!/bin/bash
# round 4: tiled-pool NCHW lookup test + reference-layout bench, Cholesky chain
# timelines (profiling build), then the HIP-graph replay of update(): the bitwise
# unit test first, the trajectory with replay on last
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04f"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -k "alt2" -v --timeout 240 --timeout-method thread > "$O/pytest_alt.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_alt.txt" | head; tail -2 "$O/pytest_alt.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/alt_time.py > "$O/alt_time.txt" 2>&1 || { tail -20 "$O/alt_time.txt"; exit 1; }
cat "$O/alt_time.txt"
timeout -k 10 500 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_update.py tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "not graph_replay" > "$O/pytest_corr_update.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_corr_update.txt" | head; tail -2 "$O/pytest_corr_update.txt"; [ $rc -eq 0 ] || exit $rc
for ab in 0 1 4 8; do
  DROID_VOL_VARIANT=2 DROID_VOL_ABLATE=$ab VOL_EDGES=1024 timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol2_ablate$ab.txt" 2>&1 || { tail -20 "$O/vol2_ablate$ab.txt"; exit 1; }
  echo "v2 ablate $ab (1024 edges)"; grep variant "$O/vol2_ablate$ab.txt"
done
timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout.json" 2> "$O/bench_reflayout.err" || { tail -20 "$O/bench_reflayout.err"; exit 1; }
cat "$O/bench_reflayout.json"
timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_new.txt" 2>&1 || { tail -20 "$O/ba_new.txt"; exit 1; }
cat "$O/ba_new.txt"
for v in t1 t0; do
  DROID_HIP_LIB="$R/droid-slam_amd/lib/ab/libdroid_hip_$v.so" timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_$v.txt" 2>&1 || { tail -20 "$O/ba_$v.txt"; exit 1; }
  echo "== $v"; cat "$O/ba_$v.txt"
done
for c in C3 C5; do
  timeout -k 10 300 python -u scripts/chol_timeline.py $c > "$O/timeline_$c.txt" 2>&1 || { tail -20 "$O/timeline_$c.txt"; exit 1; }
  cat "$O/timeline_$c.txt"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o r04f --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 3 > "$O/bench_c3_rocprof.json" 2> "$O/bench_c3_rocprof.err" || { tail -20 "$O/bench_c3_rocprof.err"; exit 1; }
cd "$R"
find "$O/prof_c3" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$O/r04f_c3_kernel_stats.csv"
head -25 "$O/r04f_c3_kernel_stats.csv" | cut -c1-220
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py -m gpu -k graph_replay -v --timeout 240 --timeout-method thread \
  > "$O/pytest_graph_unit.txt" 2>&1
rc=$?; tail -3 "$O/pytest_graph_unit.txt"; [ $rc -eq 0 ] || exit $rc
DROID_TEST_GRAPH_TRAJECTORY=1 timeout -k 10 400 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -v --timeout 360 --timeout-method thread \
  > "$O/pytest_graph_traj.txt" 2>&1
rc=$?; tail -3 "$O/pytest_graph_traj.txt"; [ $rc -eq 0 ] || exit $rc
for gr in 0 1; do
  DROID_UPDATE_GRAPHS=$gr timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > "$O/bench_C2_graphs$gr.json" 2> "$O/bench_C2_graphs$gr.err" || { tail -20 "$O/bench_C2_graphs$gr.err"; exit 1; }
  echo "C2 graphs=$gr"; cut -c1-300 "$O/bench_C2_graphs$gr.json"
done
