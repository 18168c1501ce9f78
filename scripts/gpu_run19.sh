#!/bin/bash
# bench breakdown + PMC of the band ZR conv
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/pmc19
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --breakdown --no-cpu-baseline > gpurun_out/bench19.json 2> gpurun_out/bench19.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench19.json; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d "$R/gpurun_out/pmc19/p$i" -o z --output-format csv -- python3 "$R/scripts/conv_bench.py" 2048 zr > "$R/gpurun_out/pmc19/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc19/p$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_counters.py" "$R/gpurun_out/pmc19" conv_band
