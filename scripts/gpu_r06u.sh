#!/bin/bash
# round 6: BA assembly - contribution records read 8 at a time (lib/vas) vs the product; parity, rocprof of the
# assembly kernel at C2 and C3, same-box C2 bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06u
mkdir -p $O
export PYTHONUNBUFFERED=1
DROID_HIP_LIB=droid-slam_amd/lib/vas/libdroid_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > $O/pytest_vas.txt 2>&1 || { tail -30 $O/pytest_vas.txt; exit 1; }
tail -1 $O/pytest_vas.txt
for v in vas prod; do
  L=droid-slam_amd/lib/vas/libdroid_hip.so; [ $v = prod ] && L=droid-slam_amd/lib/libdroid_hip.so
  (cd /tmp && export TMPDIR=/tmp && DROID_HIP_LIB="$R/$L" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$v" -o run --output-format csv -- python3 "$R/scripts/ba_bench.py" C2 C3 --reps 5 > "$R/$O/prof_$v.log" 2>&1) || exit 1
  ks=$(find "$O/prof_$v" -name '*kernel_stats.csv' | head -n 1)
  echo "== $v"; grep -E "assemble" "$ks" | cut -c1-160
done
for rep in 1 2; do
  for v in vas prod; do
    L=droid-slam_amd/lib/vas/libdroid_hip.so; [ $v = prod ] && L=droid-slam_amd/lib/libdroid_hip.so
    DROID_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > $O/bench_C2_${v}_$rep.json 2> $O/bench_C2_${v}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_C2_${v}_$rep.json $v
  done
done
