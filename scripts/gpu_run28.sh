#!/bin/bash
# Cholesky: parity tests + timeline
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_chol.py tests/test_gpu_ba.py -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest28.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest28.log | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python scripts/chol_timeline.py 1530 > gpurun_out/chol_tl.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/chol_tl.log | grep -v "^  k="; exit $rc
