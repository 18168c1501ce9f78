#!/bin/bash
# stereo (C4) update() parity + a C4 bench line
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py -k "stereo or factor_graph" > gpurun_out/pytest49.log 2>&1 || { tail -40 gpurun_out/pytest49.log; exit 1; }
tail -6 gpurun_out/pytest49.log
timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench49_c4.json 2> gpurun_out/bench49_c4.err || { tail -20 gpurun_out/bench49_c4.err; exit 1; }
cat gpurun_out/bench49_c4.json
