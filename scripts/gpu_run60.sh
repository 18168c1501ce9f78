#!/bin/bash
# experiment: factored z|r gates on the 256x256 tile vs two 384x128 tiles (DROID_ZR_TILE=384)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/conv_timeline.py 2048 zrp > gpurun_out/tl60_zrp.txt 2>&1 || { cat gpurun_out/tl60_zrp.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/tl60_zrp.txt | head -3
DROID_ZR_TILE=384 timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py -k "gru_pre or inp_frames or factor_graph" > gpurun_out/pytest60.log 2>&1 || { tail -30 gpurun_out/pytest60.log; exit 1; }
tail -1 gpurun_out/pytest60.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench60a.json 2> gpurun_out/bench60a.err || exit 1
DROID_ZR_TILE=384 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench60b.json 2> gpurun_out/bench60b.err || exit 1
python3 -c "
import json
for f in ('a','b'):
    d=json.load(open('gpurun_out/bench60%s.json'%f)); print(f, round(d['value'],2), 'it/s zr', round(d['roofline']['launch_ms'],3))"
