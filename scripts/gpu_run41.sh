#!/bin/bash
# edge-sharded update() (2 ranks on one GPU, gloo) == unsharded
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/pytest41.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pytest41.log | tail -30; exit $rc
