#!/bin/bash
# round 4 batch: volume/tests (c), benches (e), Cholesky (d); stops at the first failure
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for s in c e d; do
  echo "=== r04$s"
  bash scripts/gpu_r04$s.sh || { echo "r04$s failed"; exit 1; }
done
