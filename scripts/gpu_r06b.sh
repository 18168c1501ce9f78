#!/bin/bash
# round 6: Cholesky timeline + same-box BA A/B (no test pass)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || { cat $O/chol_timeline_C3.txt; exit 1; }
grep -v amdgpu.ids $O/chol_timeline_C3.txt
timeout -k 10 300 python -u scripts/ba_bench.py C3 --reps 9 > $O/ba_new.txt 2>&1 || exit 1
DROID_HIP_LIB=droid-slam_amd/lib/prev/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 --reps 9 > $O/ba_prev.txt 2>&1 || exit 1
grep -h "ba(itrs" $O/ba_new.txt $O/ba_prev.txt
