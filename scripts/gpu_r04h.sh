#!/bin/bash
# round 4: graph-replay diagnostics without the fault: the pool-ownership report
# at each capture, stopping (an exception, no replay) at the second capture
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04h"
mkdir -p "$O"
cd "$R"
DROID_GRAPH_DEBUG=1 DROID_GRAPH_DEBUG_STOP=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_trajectory.py::test_frontend_sequence_matches_oracle[True]" -m gpu -v -s --timeout 240 --timeout-method thread \
  > "$O/pytest_graph_pool.txt" 2>&1
grep -E "^\[update graph\]|^\[replay\]|graph debug stop|Error" "$O/pytest_graph_pool.txt" | grep -v "^\[replay\]" | cut -c1-3000 | tail -40
exit 0
