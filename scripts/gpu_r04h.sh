#!/bin/bash
# round 4: graph-replay diagnostics without the fault: the pool report and the
# check of every device pointer the captured body handed the library against
# the allocator's blocks, stopping (an exception) before the first replay
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04h"
mkdir -p "$O"
cd "$R"
DROID_TEST_GRAPH_TRAJECTORY=1 DROID_GRAPH_DEBUG=1 DROID_GRAPH_DEBUG_STOP_BEFORE_REPLAY=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -v -s --timeout 240 --timeout-method thread \
  > "$O/pytest_graph_ptrs.txt" 2>&1
grep -E "^\[update graph\]|graph debug stop|Error" "$O/pytest_graph_ptrs.txt" | cut -c1-4000 | tail -20
exit 0
