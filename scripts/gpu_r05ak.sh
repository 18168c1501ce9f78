#!/bin/bash
# same-box A/B of the round-5 late conv changes: the product library against the
# pre-change build (lib/r05pre, sources of 53455ec), C3 bench lines alternated
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/${AB_OUT:-r05ak}
mkdir -p $O
for r in 1 2 3; do
  for v in new pre; do
    if [ $v = pre ]; then L=droid-slam_amd/lib/r05pre/libdroid_hip.so; else L=droid-slam_amd/lib/libdroid_hip.so; fi
    DROID_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_${v}_$r.json $v
  done
done
