#!/bin/bash
# round 4: Cholesky chain (blocked panel + trsm(k+1,k) by forward substitution, L^-1 off the chain):
# parity tests, BA timing A/B and the chain timeline.
#   lib/ab/libdroid_hip_t0.so = panel4 with the round-3 chain (L^-1 then a GEMM for trsm(k+1,k))
#   lib/ab/libdroid_hip_p1.so = the round-3 column panel and chain
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04d"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py -m gpu -v --timeout 300 --timeout-method thread \
  > "$O/pytest.txt" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$O/pytest.txt" | head -20
tail -2 "$O/pytest.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_new.txt" 2>&1 || { tail -20 "$O/ba_new.txt"; exit 1; }
cat "$O/ba_new.txt"
for v in t0; do
  DROID_HIP_LIB="$R/droid-slam_amd/lib/ab/libdroid_hip_$v.so" timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_$v.txt" 2>&1 || { tail -20 "$O/ba_$v.txt"; exit 1; }
  echo "== $v"; cat "$O/ba_$v.txt"
done
timeout -k 10 300 python -u scripts/chol_timeline.py C3 > "$O/timeline_c3.txt" 2>&1 || { tail -20 "$O/timeline_c3.txt"; exit 1; }
cat "$O/timeline_c3.txt"
