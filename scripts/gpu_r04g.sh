#!/bin/bash
# round 4: diagnostics of the HIP-graph replay fault in the frontend trajectory
# (each update phase and side synchronised and named, DROID_GRAPH_DEBUG=1)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04g"
mkdir -p "$O"
cd "$R"
DROID_GRAPH_DEBUG=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -v -s --timeout 240 --timeout-method thread \
  > "$O/pytest_graph_traj_debug.txt" 2>&1
rc=$?
grep -E "^\[update graph\]|^\[replay\]" "$O/pytest_graph_traj_debug.txt" | tail -30
grep -E "Error|error" "$O/pytest_graph_traj_debug.txt" | head -5
exit $rc
