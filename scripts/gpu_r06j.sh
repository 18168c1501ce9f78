#!/bin/bash
# round 6: Cholesky - the L_kk store drain moved after the tall_solve alone (lib/varB) vs the kept kernel
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06j
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/varB/prof/libdroid_hip.so TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3_varB.txt 2>&1 || exit 1
grep -E "span|potrf tasks|tail,|second" $O/chol_timeline_C3_varB.txt
TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3_head.txt 2>&1 || exit 1
grep -E "span|potrf tasks|tail,|second" $O/chol_timeline_C3_head.txt
for rep in 1 2; do
  DROID_HIP_LIB=droid-slam_amd/lib/varB/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_varB_$rep.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_head_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
