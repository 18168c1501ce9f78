#!/bin/bash
# round 6: Cholesky rewrite - parity tests, same-box BA A/B vs the previous library, chain timeline
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py > $O/pytest_chol_ba.txt 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_chol_ba.txt; exit 1; }
tail -3 $O/pytest_chol_ba.txt
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_new_$rep.txt 2>&1 || exit 1
  DROID_HIP_LIB=droid-slam_amd/lib/prev/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prev_$rep.txt 2>&1 || exit 1
done
grep -h "ba(itrs" $O/ba_*.txt
timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/chol_timeline.py C5 > $O/chol_timeline_C5.txt 2>&1 || exit 1
cat $O/chol_timeline_C3.txt $O/chol_timeline_C5.txt | grep -v amdgpu.ids
