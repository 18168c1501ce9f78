#!/bin/bash
# round 4: cache-policy A/B builds - volume build (default = nt level-0/1 stores,
# v_vst0 = default-policy stores, v_poolnt = nt also in the pooling pass) and the
# update()'s lookups (v_ldnt = nt volume window loads): vol_bench, C3 bench
# (fused lookup) and the reference-layout bench, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r04y
mkdir -p $O
libp() { if [ $1 = lib ]; then echo $(pwd)/droid-slam_amd/lib/libdroid_hip.so; else echo $(pwd)/droid-slam_amd/lib/$1/libdroid_hip.so; fi; }
for v in lib v_vst0 v_poolnt lib v_vst0 v_poolnt; do
  echo "== $v" >> $O/vol.txt
  DROID_HIP_LIB=$(libp $v) timeout -k 10 300 python -u scripts/vol_bench.py >> $O/vol.txt 2>&1 || { tail -20 $O/vol.txt; exit 1; }
done
grep -v amdgpu.ids $O/vol.txt
for v in lib v_ldnt lib v_ldnt; do
  DROID_HIP_LIB=$(libp $v) timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('C3 $v', round(d['ms_per_step'],3), 'lookup', round(d['roofline_lookup']['launch_ms'],3))"
done
for v in lib v_ldnt lib v_ldnt; do
  DROID_HIP_LIB=$(libp $v) timeout -k 10 600 python -u bench.py --reference-layout --no-cpu-baseline > $O/bench_ref_$v.json 2> $O/bench_ref_$v.err || { tail -20 $O/bench_ref_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_ref_$v.json'));print('ref-layout $v', round(d['ms_per_step'],3))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; exit $rc
