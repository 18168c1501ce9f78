#!/bin/bash
# round 6: Cholesky chain start - the successor's version sampled before the tail's solve, its poll skipped
# (lib/vc); plus its diagonal tile by LDS-DMA into T0 in the tail (lib/vd); parity, timelines, same-box BA
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06o
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in vc vd; do
  DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol.py tests/test_gpu_ba.py > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
  DROID_HIP_LIB=droid-slam_amd/lib/$v/prof/libdroid_hip.so TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3_$v.txt 2>&1 || exit 1
  grep -E "span|potrf tasks|tail,|second" $O/chol_timeline_C3_$v.txt | head -4
done
for rep in 1 2; do
  for v in vc vd; do
    DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_${v}_$rep.txt 2>&1 || exit 1
  done
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prod_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
