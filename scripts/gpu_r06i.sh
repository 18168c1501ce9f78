#!/bin/bash
# round 6: Cholesky - the chained successor's diagonal tile by LDS-DMA during the last panel (L_kk drain
# unchanged); parity, C3 timeline, same-box BA A/B against the previous library (lib/head)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_chol.py tests/test_gpu_ba.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || exit 1
grep -E "span|potrf tasks|tail,|panels \(|second|back solve" $O/chol_timeline_C3.txt
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_new_$rep.txt 2>&1 || exit 1
  DROID_HIP_LIB=droid-slam_amd/lib/head/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_head_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
