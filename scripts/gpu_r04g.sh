#!/bin/bash
# round 4: volume variant 4 (levels 2-3 by a pooling pass) hash + timing + the
# corr tests on it, the reference-layout bench (tiled lookup timed), BA A/B,
# then diagnostics of the HIP-graph replay fault in the frontend trajectory
# (each update phase and side synchronised and named, DROID_GRAPH_DEBUG=1) - last
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04g"
mkdir -p "$O"
cd "$R"
for v in 2 4; do
  DROID_VOL_VARIANT=$v timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v$v.txt" 2>&1 || { tail -20 "$O/vol_v$v.txt"; exit 1; }
  grep -E "variant|hash" "$O/vol_v$v.txt"
done
DROID_VOL_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py -m gpu -v --timeout 240 --timeout-method thread > "$O/pytest_corr_v4.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_corr_v4.txt" | head; tail -2 "$O/pytest_corr_v4.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout.json" 2> "$O/bench_reflayout.err" || { tail -20 "$O/bench_reflayout.err"; exit 1; }
cut -c1-200 "$O/bench_reflayout.json"; grep -o '"roofline_lookup": {[^}]*}' "$O/bench_reflayout.json"
timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_new.txt" 2>&1 || { tail -20 "$O/ba_new.txt"; exit 1; }
cat "$O/ba_new.txt"
DROID_HIP_LIB="$R/droid-slam_amd/lib/ab/libdroid_hip_t1.so" timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_t1.txt" 2>&1 || { tail -20 "$O/ba_t1.txt"; exit 1; }
echo "== t1"; cat "$O/ba_t1.txt"
DROID_TEST_GRAPH_TRAJECTORY=1 DROID_GRAPH_DEBUG=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -v -s --timeout 240 --timeout-method thread \
  > "$O/pytest_graph_traj_debug.txt" 2>&1
rc=$?
grep -E "^\[update graph\]|^\[replay\]" "$O/pytest_graph_traj_debug.txt" | tail -30
grep -E "Error|error" "$O/pytest_graph_traj_debug.txt" | head -5
exit $rc
