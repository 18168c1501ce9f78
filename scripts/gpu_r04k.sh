#!/bin/bash
# round 4: graph replay with the BA's resets as kernels instead of runtime
# memset nodes: the unit test, then the frontend sequence with replay on
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04k"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_update.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_ba_update.txt" 2>&1
rc=$?; tail -2 "$O/pytest_ba_update.txt"; [ $rc -eq 0 ] || exit $rc
DROID_TEST_GRAPH_TRAJECTORY=1 DROID_GRAPH_DEBUG=1 timeout -k 10 400 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -x -s --timeout 360 --timeout-method thread \
  > "$O/pytest_graph_traj.txt" 2>&1
rc=$?
grep -E "^\[update graph\]" "$O/pytest_graph_traj.txt" | grep -v "pointers captured" | tail -6 | cut -c1-300
grep -E "passed|failed|illegal" "$O/pytest_graph_traj.txt" | tail -3
exit $rc
