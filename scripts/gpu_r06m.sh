#!/bin/bash
# round 6: BA linearisation kernels - the edge Hessian two pixels ahead, the frame Schur kernel with every
# edge's inputs issued up front (lib/varBA) vs the product library; parity and same-box BA timing
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06m
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/varBA/libdroid_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_chol.py > $O/pytest_varBA.txt 2>&1 || { tail -30 $O/pytest_varBA.txt; exit 1; }
tail -1 $O/pytest_varBA.txt
for rep in 1 2; do
  DROID_HIP_LIB=droid-slam_amd/lib/varBA/libdroid_hip.so timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_varBA_$rep.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 7 > $O/ba_prod_$rep.txt 2>&1 || exit 1
done
grep "ba(itrs" $O/ba_*.txt
(cd /tmp && export TMPDIR=/tmp && DROID_HIP_LIB="$R/droid-slam_amd/lib/varBA/libdroid_hip.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/scripts/ba_bench.py" C3 --reps 5 > "$R/$O/prof.log" 2>&1) || exit 1
ks=$(find "$O/prof" -name '*kernel_stats.csv' | head -n 1)
grep -E "hessian|schur|chol" "$ks" | cut -c1-200
