#!/bin/bash
# round 6: Cholesky timeline only (profiling build)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06c
mkdir -p $O
export PYTHONUNBUFFERED=1
TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || { cat $O/chol_timeline_C3.txt; exit 1; }
grep -v amdgpu.ids $O/chol_timeline_C3.txt
