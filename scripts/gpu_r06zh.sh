#!/bin/bash
# round 6: z|r 256x256 tile with the per-frame term loaded before pass 1 (kEarlyPre) vs lib/cur
# (loaded after pass 1): digests + time, the conv / update GPU tests, the timeline,
# then the C3 bench alternating
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06zh
mkdir -p $O
export PYTHONUNBUFFERED=1
CUR=droid-slam_amd/lib/cur/libdroid_hip.so
NEW=droid-slam_amd/lib/libdroid_hip.so
for rep in 1 2; do
  DROID_HIP_LIB=$CUR timeout -k 10 120 python -u scripts/zr_ab.py 2048 2>&1 | grep -v amdgpu.ids || exit 1
  DROID_HIP_LIB=$NEW timeout -k 10 120 python -u scripts/zr_ab.py 2048 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_conv_c3.py tests/test_gpu_conv_tiles.py tests/test_gpu_update_full.py tests/test_gpu_update.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 120 python -u scripts/conv_timeline.py 2048 zrp > $O/tl_zrp.txt 2>&1 || { tail -5 $O/tl_zrp.txt; exit 1; }
grep -v amdgpu.ids $O/tl_zrp.txt
for rep in 1 2; do
  for v in cur new; do
    L=$NEW; [ $v = cur ] && L=$CUR
    DROID_HIP_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_C3_${v}_$rep.json 2> $O/bench_C3_${v}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], round(d['value'],3), round(d['ms_per_step'],3), 'zr', round(d['roofline']['launch_ms'],3))" $O/bench_C3_${v}_$rep.json $v
  done
done
