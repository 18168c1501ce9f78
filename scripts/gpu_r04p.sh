#!/bin/bash
# round 4: potrf chains + kLinv (Cholesky critical chain) - parity tests, BA timing
# with the chains on and off, and the C3 / C5 Cholesky timelines (profiling build)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04p"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > "$O/pytest_chol_ba.txt" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$O/pytest_chol_ba.txt" | head; tail -1 "$O/pytest_chol_ba.txt"; [ $rc -eq 0 ] || exit $rc
for ch in 2 1 0 2; do
  DROID_CHOL_CHAIN=$ch timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > "$O/ba_chain$ch.txt" 2>&1 || { tail -20 "$O/ba_chain$ch.txt"; exit 1; }
  echo "chain=$ch"; grep ba "$O/ba_chain$ch.txt"
done
for c in C3 C5; do
  timeout -k 10 300 python -u scripts/chol_timeline.py $c > "$O/timeline_$c.txt" 2>&1 || { tail -20 "$O/timeline_$c.txt"; exit 1; }
  head -8 "$O/timeline_$c.txt"
done
