#!/bin/bash
# packed (lower-triangle + rhs) all-reduce of the reduced system: sharded parity, 2-rank bench rehearsal
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_gpu_ba.py > gpurun_out/pytest61.log 2>&1 || { tail -40 gpurun_out/pytest61.log; exit 1; }
tail -3 gpurun_out/pytest61.log
DROID_BENCH_ONE_DEVICE=1 DROID_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench61_2rank.json 2> gpurun_out/bench61_2rank.err || { grep -v amdgpu.ids gpurun_out/bench61_2rank.err | tail -20; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench61_2rank.json')); print('2-rank', round(d['value'],2), d['state_finite'])"
