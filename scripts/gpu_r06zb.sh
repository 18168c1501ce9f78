#!/bin/bash
# round 6: DWHEAD pass 1 with the column biases read up front and immediate store offsets (lib/cur = the v2 epilogue) on one box:
# bitwise head output, time, the conv/fused GPU tests, the timeline
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06zb
mkdir -p $O
export PYTHONUNBUFFERED=1
CUR=droid-slam_amd/lib/cur/libdroid_hip.so
NEW=droid-slam_amd/lib/libdroid_hip.so
for rep in 1 2; do
  DROID_HIP_LIB=$CUR timeout -k 10 120 python -u scripts/dwh_ab.py 2048 /tmp/head_cur.npy || exit 1
  DROID_HIP_LIB=$NEW timeout -k 10 120 python -u scripts/dwh_ab.py 2048 /tmp/head_new.npy || exit 1
done
python3 -c "
import numpy as np
a=np.load('/tmp/head_cur.npy'); b=np.load('/tmp/head_new.npy')
print('bitwise equal:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max|d|', float(np.abs(a-b).max()), 'n diff', int((a!=b).sum()))
" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_conv_c3.py tests/test_gpu_conv_tiles.py tests/test_gpu_update_full.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 120 python -u scripts/conv_timeline.py 2048 dwh > $O/tl_dwh.txt 2>&1 || { tail -5 $O/tl_dwh.txt; exit 1; }
cat $O/tl_dwh.txt
