#!/bin/bash
# SQ counters of the on-demand lookup's corr_alt2_kernel variants (A/B build:
# scripts/alt_time.py --quick runs every variant on the C3 coordinates), one
# rocprofv3 --pmc run per pass (<= 8 SQ counters), summarised per kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmcalt}; mkdir -p $O
export DROID_HIP_LIB=$R/droid-slam_amd/lib/ab/libdroid_hip.so
n=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/p$n -o run --output-format csv -- python3 $R/scripts/alt_time.py --quick > $O/p$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p$n.log; exit $rc; }
  python3 $R/scripts/pmc_counters.py $O/p$n corr_alt > $O/p${n}_summary.txt
  cat $O/p${n}_summary.txt
done
