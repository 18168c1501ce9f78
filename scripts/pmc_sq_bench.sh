#!/bin/bash
# SQ counter passes over a short C3 bench (every update-path kernel), one
# rocprofv3 --pmc run per pass (<= 8 SQ counters each), summarised per kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmcsq}; mkdir -p $O
shift
n=0
for pass in "$@"; do
  n=$((n + 1))
  timeout -s KILL 150 rocprofv3 --pmc $pass -d $O/p$n -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/p$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $R/scripts/pmc_counters.py $O/p$n > $O/p${n}_summary.txt
done
