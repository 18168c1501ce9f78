#!/bin/bash
# HBM traffic per launch from separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md §HBM)
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/pmc_traffic"
sha256sum "$R/droid-slam_amd/lib/libdroid_hip.so" | cut -c1-16 > "$R/gpurun_out/pmc_traffic/lib_sha16.txt"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_traffic/$c" -o w --output-format csv -- python3 "$R/scripts/pmc_workload.py" > "$R/gpurun_out/pmc_traffic/$c.log" 2>&1 || exit 1
done
# the records land in profiles/ on the box AND under gpurun_out/ (merged back by gpurun;
# locally: python3 scripts/pmc_summarize.py gpurun_out/pmc_traffic profiles)
mkdir -p "$R/gpurun_out/pmc_traffic/profiles"
python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out/pmc_traffic" "$R/gpurun_out/pmc_traffic/profiles" &&
python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out/pmc_traffic" "$R/profiles"
