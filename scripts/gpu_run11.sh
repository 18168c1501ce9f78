#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
for h in 0 4; do
  export DROID_CONV_HALO=$h
  timeout -k 10 300 rocprofv3 --pmc $P1 -d "$R/gpurun_out/pmc/h${h}_p1" -o zr --output-format csv -- python3 "$R/scripts/conv_bench.py" 2048 zr > "$R/gpurun_out/pmc/h${h}_p1.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $P2 -d "$R/gpurun_out/pmc/h${h}_p2" -o zr --output-format csv -- python3 "$R/scripts/conv_bench.py" 2048 zr > "$R/gpurun_out/pmc/h${h}_p2.log" 2>&1 || exit 1
done
echo done
