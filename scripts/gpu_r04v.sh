#!/bin/bash
# round 4: the motion / global-context branches on a side stream (DROID_BRANCH_STREAMS)
# - update-path tests, then C3 / C2 / C5 benches with the side stream off and on, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_update.py tests/test_gpu_update_full.py \
  tests/test_gpu_trajectory.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/pytest.txt | head; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C2; do
  for bs in 0 1 0 1; do
    DROID_BRANCH_STREAMS=$bs timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline > $O/bench_${cfg}_bs$bs.json 2> $O/bench_${cfg}_bs$bs.err || { tail -20 $O/bench_${cfg}_bs$bs.err; exit 1; }
    echo "$cfg branch_streams=$bs $(cut -c1-160 $O/bench_${cfg}_bs$bs.json | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*')"
  done
done
for bs in 0 1; do
  DROID_BRANCH_STREAMS=$bs timeout -k 10 600 python -u bench.py --config C5 --no-cpu-baseline > $O/bench_C5_bs$bs.json 2> $O/bench_C5_bs$bs.err || { tail -20 $O/bench_C5_bs$bs.err; exit 1; }
  echo "C5 branch_streams=$bs $(grep -o '"ms_per_step": [0-9.]*' $O/bench_C5_bs$bs.json)"
done
