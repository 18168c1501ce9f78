#!/bin/bash
# round 6: cleaned Cholesky - BA/Cholesky/sharded GPU tests, C3 bench, 2-rank (gloo, one device) and RCCL 1-rank bench lines
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_chol.py tests/test_gpu_ba.py tests/test_gpu_ba_scale.py tests/test_gpu_sharded.py tests/test_gpu_trajectory.py tests/test_gpu_fused.py::test_reference_layout_module_inference_refill_in_place tests/test_gpu_fused.py::test_reference_layout_module_under_inference_mode > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3.json')); print('C3', d['value'], d['ms_per_step'])"
timeout -k 10 500 env DROID_BENCH_ONE_DEVICE=1 DROID_BENCH_BACKEND=gloo python -u bench.py --gpus 2 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.loads([x for x in open('$O/bench_2rank.json') if x.startswith('{')][-1]); print('2rank', d['value'], d.get('allreduce'), d.get('serial'))"
timeout -k 10 400 env DROID_BENCH_FORCE_DIST=1 python -u bench.py --no-cpu-baseline > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { tail -20 $O/bench_rccl1.err; exit 1; }
python3 -c "import json; d=json.loads([x for x in open('$O/bench_rccl1.json') if x.startswith('{')][-1]); print('rccl1', d['value'], d.get('allreduce'), d.get('serial'))"
