#!/bin/bash
# round 4: pool23 two-values-per-lane (volume build bytes + timing), flow_enc0 256-pixel
# tiles (parity + C3 timing, 128 vs 256), then the C3 bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04r"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_fused.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest_corr_fused.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_corr_fused.txt" | head; tail -1 "$O/pytest_corr_fused.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v4.txt" 2>&1 || { tail -20 "$O/vol_v4.txt"; exit 1; }
cat "$O/vol_v4.txt"
for tp in 128 256; do
  DROID_FE_TP=$tp timeout -k 10 300 python -u scripts/fe_bench.py > "$O/fe_tp$tp.txt" 2>&1 || { tail -20 "$O/fe_tp$tp.txt"; exit 1; }
  cat "$O/fe_tp$tp.txt"
done
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cut -c1-300 "$O/bench.json"
