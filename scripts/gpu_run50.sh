#!/bin/bash
# gate convs with the inp term per source frame: parity + bench breakdown + kernel stats
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out; R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_update.py > gpurun_out/pytest50.log 2>&1 || { tail -40 gpurun_out/pytest50.log; exit 1; }
tail -2 gpurun_out/pytest50.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof50" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --breakdown --no-cpu-baseline > "$R/gpurun_out/bench50.json" 2> "$R/gpurun_out/bench50.err" || exit 1
cd "$R"; python3 -c "import json; d=json.load(open('gpurun_out/bench50.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'], d['roofline']['frac'], d['roofline']['launch_ms'])"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench50_clean.json 2> gpurun_out/bench50_clean.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench50_clean.json')); print('clean', round(d['value'],2), 'it/s')"
