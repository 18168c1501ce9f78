#!/bin/bash
# SQ counters of the Q band conv, lock-step vs ping-pong
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p "$R/gpurun_out/pmc_q"
cd /tmp && export TMPDIR=/tmp
for pp in 0 1; do
DROID_CONV_PP=$pp timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d "$R/gpurun_out/pmc_q/pp$pp" -o a --output-format csv -- python3 "$R/scripts/conv_bench.py" 1024 q > "$R/gpurun_out/pmc_q/pp$pp.log" 2>&1 || exit 1
cd "$R"; echo "== PP=$pp"; python3 scripts/pmc_counters.py gpurun_out/pmc_q/pp$pp band; cd /tmp
done
