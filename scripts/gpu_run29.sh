#!/bin/bash
# SQ counters of the band ZR conv (stall anatomy)
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p "$R/gpurun_out/pmc_zr"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES -d "$R/gpurun_out/pmc_zr/a" -o a --output-format csv -- python3 "$R/scripts/conv_bench.py" 1024 zr > "$R/gpurun_out/pmc_zr/a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -d "$R/gpurun_out/pmc_zr/b" -o b --output-format csv -- python3 "$R/scripts/conv_bench.py" 1024 zr > "$R/gpurun_out/pmc_zr/b.log" 2>&1 || exit 1
cd "$R"; python3 scripts/pmc_counters.py gpurun_out/pmc_zr band
