#!/bin/bash
# Rehearse bench.py's 2-rank path on a one-GPU box (both ranks on cuda:0, gloo collectives).
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
DROID_BENCH_ONE_DEVICE=1 DROID_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err; rc=$?
echo "2-rank rc=$rc"; cat gpurun_out/bench_2rank.json; grep -v amdgpu.ids gpurun_out/bench_2rank.err | tail -8
exit $rc
