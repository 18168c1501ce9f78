#!/bin/bash
# round 4: blocked Cholesky panel - parity tests and BA timing A/B (lib/ab/libdroid_hip_p1.so = the old panel)
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
timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_panel4.txt" 2>&1 || { tail -20 "$O/ba_panel4.txt"; exit 1; }
cat "$O/ba_panel4.txt"
DROID_HIP_LIB="$R/droid-slam_amd/lib/ab/libdroid_hip_p1.so" timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 > "$O/ba_panel1.txt" 2>&1 || { tail -20 "$O/ba_panel1.txt"; exit 1; }
cat "$O/ba_panel1.txt"
