#!/bin/bash
# round 6: back solve - two granule polls in flight (lib/vg) vs the product; parity, timeline, same-box BA
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06s
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/vg/libdroid_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol.py tests/test_gpu_ba.py > $O/pytest_vg.txt 2>&1 || { tail -30 $O/pytest_vg.txt; exit 1; }
tail -1 $O/pytest_vg.txt
for v in vg prof; do
  L=droid-slam_amd/lib/$v/prof/libdroid_hip.so; [ $v = prof ] && L=droid-slam_amd/lib/prof/libdroid_hip.so
  DROID_HIP_LIB=$L TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "span|back solve" $O/chol_timeline_C3_$v.txt | head -3
done
for rep in 1 2; do
  DROID_HIP_LIB=droid-slam_amd/lib/vg/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_vg_$rep.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prod_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
