#!/bin/bash
# round 6: Cholesky worker count by task-graph size (product library) - BA tests, then
# BA(itrs=2) at C3 / C5 against lib/cur (one worker per two CUs), alternating
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06ze
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ba_scale.py tests/test_gpu_chol.py tests/test_gpu_sharded.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for rep in 1 2; do
  for v in cur new; do
    L=droid-slam_amd/lib/libdroid_hip.so; [ $v = cur ] && L=droid-slam_amd/lib/cur/libdroid_hip.so
    echo "== $v"
    DROID_HIP_LIB=$L timeout -k 10 300 python -u scripts/ba_bench.py C3 C5 --reps 8 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
