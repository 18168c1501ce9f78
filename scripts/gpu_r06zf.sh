#!/bin/bash
# round 6: Cholesky timelines at C3 / C5 with the new worker count (profiling build)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06zf
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/chol_timeline.py C3 > $O/tl_C3.txt 2>&1 || { tail -20 $O/tl_C3.txt; exit 1; }
head -12 $O/tl_C3.txt
timeout -k 10 300 python -u scripts/chol_timeline.py C5 > $O/tl_C5.txt 2>&1 || { tail -20 $O/tl_C5.txt; exit 1; }
head -12 $O/tl_C5.txt
