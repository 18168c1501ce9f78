#!/bin/bash
# SQ counters of the z|r gate conv on both 256x256 tiles (scripts/zr_tiles.py:
# 8-wave band tile, 4-wave tile), one rocprofv3 --pmc pass, summarised per kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmczr}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run --output-format csv -- python3 $R/scripts/zr_tiles.py > $O/p1.log 2>&1
rc=$?; echo "pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/scripts/pmc_counters.py $O/p1 conv_band > $O/p1_summary.txt; cat $O/p1_summary.txt
