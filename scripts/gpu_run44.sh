#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --breakdown --no-cpu-baseline > gpurun_out/bench44.json 2> gpurun_out/bench44.err || { tail -5 gpurun_out/bench44.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench44.json')); print(round(d['value'],2), 'it/s', d['breakdown_ms'], d['roofline']['launch_ms'], d['iteration_roofline'])"
