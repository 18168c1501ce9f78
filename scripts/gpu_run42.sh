#!/bin/bash
# band conv timeline (profiling build): prologue / loop / epilogue / inter-workgroup gap
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1
for c in q ce2 zr; do timeout -k 10 120 python scripts/conv_timeline.py 2048 $c 2>&1 | grep -v amdgpu || exit 1; done
