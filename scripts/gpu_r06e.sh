#!/bin/bash
# round 6: full GPU suite on the split boundary (testing hooks in lib/ab only), smoke, Cholesky tail timeline
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
TL_BCOL=1 timeout -k 10 300 python -u scripts/chol_timeline.py C3 > $O/chol_timeline_C3.txt 2>&1 || exit 1
grep -E "span|potrf tasks|tail,|panels \(|second|back solve" $O/chol_timeline_C3.txt
