#!/bin/bash
# round 6: BA linearisation kernels one change at a time - the edge Hessian two pixels ahead (lib/varH), the
# frame Schur kernel with every edge's inputs issued up front (lib/varSc); parity, then same-box BA timing
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06n
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in varH varSc; do
  DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > $O/pytest_$v.txt 2>&1
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
for rep in 1 2; do
  for v in varH varSc; do
    DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_${v}_$rep.txt 2>&1 || exit 1
  done
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prod_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
