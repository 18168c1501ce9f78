#!/bin/bash
# ping-pong band conv A/B
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export PYTHONUNBUFFERED=1
for cfg in "0 1" "1 1" "1 2" "0 2"; do set -- $cfg
  echo "== PP=$1 BAND=$2"
  DROID_CONV_PP=$1 DROID_CONV_BAND=$2 timeout -k 10 120 python scripts/conv_bench.py 2048 2>&1 | grep -v amdgpu || exit 1
done
