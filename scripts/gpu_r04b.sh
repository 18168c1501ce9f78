#!/bin/bash
# round 4: touched tests (conv tiles at C3 shape, inference mode, sharded status, lowmem BA spy)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04b"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv_c3.py tests/test_gpu_fused.py tests/test_gpu_update.py \
  tests/test_gpu_ba_scale.py tests/test_gpu_sharded.py -m gpu -v --timeout 300 --timeout-method thread \
  > "$O/pytest.txt" 2>&1
rc=$?
tail -25 "$O/pytest.txt"
exit $rc
