#!/bin/bash
# PMC: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the ZR conv and the new fused lookup;
# SQ stall anatomy of the fused lookup
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out/pmc_traffic gpurun_out/pmc_ce0
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_traffic/$c" -o w --output-format csv -- python3 "$R/scripts/pmc_workload.py" > "$R/gpurun_out/pmc_traffic/$c.log" 2>&1 || exit 1
done
python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out/pmc_traffic" "$R/gpurun_out/pmc_traffic" || exit 1   # copied to profiles/ here
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d "$R/gpurun_out/pmc_ce0/a" -o a --output-format csv -- python3 "$R/scripts/pmc_workload.py" > "$R/gpurun_out/pmc_ce0/a.log" 2>&1 || exit 1
cd "$R"; python3 scripts/pmc_counters.py gpurun_out/pmc_ce0 corr_ce0
