set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03bf; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/counters.txt | sort -u > $O/sq_names.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run --output-format csv -- python3 $R/scripts/wino_bench.py 2048 zr > $O/p1.log 2>&1
echo p1 rc=$?
python3 $R/scripts/pmc_counters.py $O/p1 conv_ > $O/p1_summary.txt; cat $O/p1_summary.txt
