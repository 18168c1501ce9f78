#!/bin/bash
# round 6 (after the head epilogue and the Cholesky worker count): the round's end-to-end change on one box - C3 bench with the round-start library (lib/prev) and
# the final library, alternating, two runs each
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06xb
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in prev final; do
    L=droid-slam_amd/lib/libdroid_hip.so; [ $v = prev ] && L=droid-slam_amd/lib/prev/libdroid_hip.so
    DROID_HIP_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_C3_${v}_$rep.json 2> $O/bench_C3_${v}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], round(d['value'],3), round(d['ms_per_step'],3), 'zr', round(d['roofline']['launch_ms'],3))" $O/bench_C3_${v}_$rep.json $v
  done
done
