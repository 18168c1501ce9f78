#!/bin/bash
# round 4: the C3-shape gate-conv parity tests under a rocprofv3 kernel trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04a"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 -u -m pytest "$R/tests/test_gpu_conv_c3.py" -v --rootdir "$R" --timeout 300 --timeout-method thread \
  > "$O/pytest_conv_c3.txt" 2>&1
rc=$?
tail -15 "$O/pytest_conv_c3.txt"
ks=$(find "$O/prof" -name '*kernel_stats.csv' | head -n 1)
[ -n "$ks" ] && cp "$ks" "$O/kernel_stats.csv" && grep -E "conv_band" "$O/kernel_stats.csv" | cut -c1-200
exit $rc
