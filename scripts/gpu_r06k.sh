#!/bin/bash
# round 6: Cholesky stores - batched LDS reads before the stores of L_kk and of full tiles (lib/varS), the same
# with the L_kk drain after the tall_solve (lib/varS2), against the kept kernel (lib/libdroid_hip.so)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06k
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/varS/libdroid_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol.py tests/test_gpu_ba.py > $O/pytest_varS.txt 2>&1 || { tail -30 $O/pytest_varS.txt; exit 1; }
tail -1 $O/pytest_varS.txt
for v in varS varS2; do
  DROID_HIP_LIB=droid-slam_amd/lib/$v/prof/libdroid_hip.so TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "span|potrf tasks|tail,|second" $O/chol_timeline_C3_$v.txt | head -4
done
for rep in 1 2; do
  for v in varS varS2; do
    DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_${v}_$rep.txt 2>&1 || exit 1
  done
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_head_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
