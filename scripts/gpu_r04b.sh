#!/bin/bash
# round 4: touched tests + volume-build A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04b"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u scripts/gate_tiles.py > "$O/gate_tiles.txt" 2>&1 || { tail -20 "$O/gate_tiles.txt"; exit 1; }
cat "$O/gate_tiles.txt"
timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v2.txt" 2>&1 || { tail -20 "$O/vol_v2.txt"; exit 1; }
cat "$O/vol_v2.txt"
DROID_VOL_V1=1 timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v1.txt" 2>&1 || { tail -20 "$O/vol_v1.txt"; exit 1; }
cat "$O/vol_v1.txt"
timeout -k 10 1100 python -u -m pytest tests/test_gpu_conv_c3.py tests/test_gpu_fused.py tests/test_gpu_update.py \
  tests/test_gpu_corr.py tests/test_gpu_ba_scale.py tests/test_gpu_sharded.py -m gpu -v --timeout 300 --timeout-method thread \
  > "$O/pytest.txt" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" "$O/pytest.txt" | grep -v PASSED | head -20
tail -3 "$O/pytest.txt"
exit $rc
