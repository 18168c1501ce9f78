#!/bin/bash
# round 4: graph replay confirmation (frontend sequence again, C2 bench with /
# without replay), then the full GPU suite, smoke and the default bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04l"
mkdir -p "$O"
cd "$R"
DROID_TEST_GRAPH_TRAJECTORY=1 timeout -k 10 400 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -x -q --timeout 360 --timeout-method thread \
  > "$O/pytest_graph_traj.txt" 2>&1
rc=$?; tail -1 "$O/pytest_graph_traj.txt"; [ $rc -eq 0 ] || exit $rc
for gr in 0 1; do
  DROID_UPDATE_GRAPHS=$gr timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > "$O/bench_C2_graphs$gr.json" 2> "$O/bench_C2_graphs$gr.err" || { tail -20 "$O/bench_C2_graphs$gr.err"; exit 1; }
  echo "C2 graphs=$gr"; cut -c1-260 "$O/bench_C2_graphs$gr.json"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu_all.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_gpu_all.txt" | head; tail -1 "$O/pytest_gpu_all.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -20 "$O/smoke.txt"; exit 1; }
tail -2 "$O/smoke.txt"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cut -c1-400 "$O/bench.json"
