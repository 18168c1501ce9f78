#!/bin/bash
# round 6: the dataflow Cholesky's worker count re-measured (round 2 chose one per two CUs)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=${O:-gpurun_out/r06zc}
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so timeout -k 10 300 python -u scripts/chol_grid_ab.py C3 --grids 0 160 192 224 256 320 --reps 8 > $O/grid_C3.txt 2>&1 || { tail -20 $O/grid_C3.txt; exit 1; }
cat $O/grid_C3.txt
DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so timeout -k 10 400 python -u scripts/chol_grid_ab.py C5 --grids 0 160 176 192 208 224 --reps 4 > $O/grid_C5.txt 2>&1 || { tail -20 $O/grid_C5.txt; exit 1; }
cat $O/grid_C5.txt
