#!/bin/bash
# PMC counters of the band conv (z|r shape): stall breakdown, LDS, MFMA busy.
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/pmc18"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc18/counters.txt" 2>&1
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d "$R/gpurun_out/pmc18/p$i" -o z --output-format csv -- python3 "$R/scripts/conv_bench.py" 2048 zr > "$R/gpurun_out/pmc18/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc18/p$i.log"; }
done
python3 "$R/scripts/pmc_counters.py" "$R/gpurun_out/pmc18" conv_band
