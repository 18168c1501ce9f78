#!/bin/bash
# round 4: the volume build's store cache policy (DROID_VOL_STORE_AUX A/B builds:
# 0 default, 2 nt, 16 sc1, 18 nt|sc1), alternating, bytes hashed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r04x
mkdir -p $O
for rep in 1 2; do
  for v in lib v_vst2 v_vst16 v_vst18; do
    if [ $v = lib ]; then L=droid-slam_amd/lib/libdroid_hip.so; else L=droid-slam_amd/lib/$v/libdroid_hip.so; fi
    echo "== $v" >> $O/vol_aux.txt
    DROID_HIP_LIB=$(pwd)/$L timeout -k 10 300 python -u scripts/vol_bench.py >> $O/vol_aux.txt 2>&1 || { tail -20 $O/vol_aux.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/vol_aux.txt
