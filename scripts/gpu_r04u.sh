#!/bin/bash
# round 4: DROID_ZDEFER A/B (gate timing + h' bytes, alternating builds), the
# gate / update tests, and the C3 bench on the default (deferred) build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r04u
mkdir -p $O
for lib in lib v_zd0 lib v_zd0; do
  if [ $lib = lib ]; then L=droid-slam_amd/lib/libdroid_hip.so; else L=droid-slam_amd/lib/$lib/libdroid_hip.so; fi
  DROID_HIP_LIB=$(pwd)/$L timeout -k 10 300 python -u scripts/zdefer_ab.py >> $O/zdefer_ab.txt 2>&1 || { tail -20 $O/zdefer_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/zdefer_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_conv_c3.py tests/test_gpu_conv_tiles.py \
  tests/test_gpu_update.py tests/test_gpu_update_full.py tests/test_gpu_trajectory.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/pytest.txt | head; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
