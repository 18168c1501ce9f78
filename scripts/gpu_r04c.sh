#!/bin/bash
# round 4: volume-build ablations, gate tiles, the touched tests, bench C3 + reference layout
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04c"
mkdir -p "$O"
cd "$R"
for v in 1 2 3; do
  DROID_VOL_VARIANT=$v timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v$v.txt" 2>&1 || { tail -20 "$O/vol_v$v.txt"; exit 1; }
  grep -E "variant|hash" "$O/vol_v$v.txt"
done
for ab in 1 2; do
  DROID_VOL_ABLATE=$ab VOL_EDGES=1024 timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_ablate$ab.txt" 2>&1 || { tail -20 "$O/vol_ablate$ab.txt"; exit 1; }
  echo "ablate $ab (1024 edges)"; grep variant "$O/vol_ablate$ab.txt"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_c3.py tests/test_gpu_fused.py tests/test_gpu_corr.py -m gpu -v --timeout 300 --timeout-method thread \
  > "$O/pytest.txt" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$O/pytest.txt" | head -20
tail -2 "$O/pytest.txt"
[ $rc -eq 0 ] || exit $rc
