#!/bin/bash
# band conv main-loop ablations (profiling builds; timing only)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1
for v in prof abl4 abl2; do
  echo "=== $v"
  for c in q ce2; do DROID_HIP_LIB=droid-slam_amd/lib/$v/libdroid_hip.so timeout -k 10 120 python scripts/conv_timeline.py 2048 $c 2>&1 | grep -E "^q|^ce2|main loop|epilogue issue|prologue" || exit 1; done
done
