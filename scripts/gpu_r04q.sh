#!/bin/bash
# round 4: the reference-layout drop-in bench (cooperative NCHW lookup on / off),
# the correlation-volume build (variant 4 with the pooling pass) and the C3 bench
# with the Cholesky chains on / off
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04q"
mkdir -p "$O"
cd "$R"
for co in 1 0; do
  DROID_LOOKUP_COOP=$co timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > "$O/bench_reflayout_coop$co.json" 2> "$O/bench_reflayout_coop$co.err" || { tail -20 "$O/bench_reflayout_coop$co.err"; exit 1; }
  echo "coop=$co"; cut -c1-200 "$O/bench_reflayout_coop$co.json"
done
for v in 4 2; do
  DROID_VOL_VARIANT=$v timeout -k 10 300 python -u scripts/vol_bench.py > "$O/vol_v$v.txt" 2>&1 || { tail -20 "$O/vol_v$v.txt"; exit 1; }
  echo "vol v$v"; tail -3 "$O/vol_v$v.txt"
done
for ch in 1 2; do
  DROID_CHOL_CHAIN=$ch timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$O/bench_chain$ch.json" 2> "$O/bench_chain$ch.err" || { tail -20 "$O/bench_chain$ch.err"; exit 1; }
  echo "chain=$ch"; cut -c1-200 "$O/bench_chain$ch.json"
done
