#!/bin/bash
# round 4: cache-policy A/B builds on the update path - v_epint (band epilogue
# stores nt), v_glont (gru_glo's stream nt), v_bandant (band conv input bands nt):
# the C3 bench step, z|r launch and fused-lookup launch per build, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r04z
mkdir -p $O
libp() { if [ $1 = lib ]; then echo $(pwd)/droid-slam_amd/lib/libdroid_hip.so; else echo $(pwd)/droid-slam_amd/lib/$1/libdroid_hip.so; fi; }
for rep in 1 2; do
  for v in lib v_epint v_glont v_bandant; do
    DROID_HIP_LIB=$(libp $v) timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -20 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('C3 $v', round(d['ms_per_step'],3), 'zr', round(d['roofline']['launch_ms'],3), 'lookup', round(d['roofline_lookup']['launch_ms'],3))"
  done
done
