#!/bin/bash
# One parameterised GPU-box runner (run through gpurun from the repo root):
#   bash scripts/gpu_check.sh TAG STEP [STEP ...]
# Steps, run in the order given, each under its own time limit, stopping at
# the first failure: tests | tests:<pytest -k expr> | smoke | rocprof | pmc |
# bench | bench:<config> | rank2 | py:<script.py args...>
# Output goes to gpurun_out/TAG/.
set -o pipefail
TAG="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
export DROID_REPORT_DIR="$R/gpurun_out/$TAG"
O="gpurun_out/$TAG"
PYN=0
mkdir -p "$O"

fail() { echo "step $1 failed (rc=$2)"; tail -40 "$3"; exit "$2"; }

for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
        > "$O/pytest_gpu.txt" 2>&1 || fail "$step" $? "$O/pytest_gpu.txt"
      tail -3 "$O/pytest_gpu.txt" ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
        -k "${step#tests:}" > "$O/pytest_sel.txt" 2>&1 || fail "$step" $? "$O/pytest_sel.txt"
      tail -3 "$O/pytest_sel.txt" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 \
        || fail "$step" $? "$O/smoke.txt"
      tail -1 "$O/smoke.txt" ;;
    rocprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" \
        -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
        > "$R/$O/bench_rocprof.json" 2> "$R/$O/bench_rocprof.err") || fail "$step" $? "$O/bench_rocprof.err"
      ks=$(find "$O/prof" -name '*kernel_stats.csv' | head -n 1)
      cp "$ks" "$O/rocprof_kernel_stats.csv"
      python3 scripts/kstats.py "$O/bench_rocprof.json" "$O/rocprof_kernel_stats.csv" > "$O/rocprof_top.txt"
      head -30 "$O/rocprof_top.txt" ;;
    rocprof:*)
      c="${step#rocprof:}"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$c" \
        -o run --output-format csv -- python3 "$R/bench.py" --config "$c" --steps 10 --warmup 3 --no-cpu-baseline \
        > "$R/$O/bench_rocprof_$c.json" 2> "$R/$O/bench_rocprof_$c.err") || fail "$step" $? "$O/bench_rocprof_$c.err"
      ks=$(find "$O/prof_$c" -name '*kernel_stats.csv' | head -n 1)
      cp "$ks" "$O/rocprof_kernel_stats_$c.csv"
      python3 scripts/kstats.py "$O/bench_rocprof_$c.json" "$O/rocprof_kernel_stats_$c.csv" > "$O/rocprof_top_$c.txt"
      head -40 "$O/rocprof_top_$c.txt" ;;
    pmc)
      timeout -k 10 900 bash scripts/pmc_traffic.sh > "$O/pmc.log" 2>&1 || fail "$step" $? "$O/pmc.log"
      tail -3 "$O/pmc.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || fail "$step" $? "$O/bench.err"
      cat "$O/bench.json" ;;
    bench:*)
      c="${step#bench:}"
      timeout -k 10 600 python -u bench.py --config "$c" --no-cpu-baseline > "$O/bench_$c.json" \
        2> "$O/bench_$c.err" || fail "$step" $? "$O/bench_$c.err"
      cat "$O/bench_$c.json" ;;
    rank2)
      # bench.py's 2-rank path rehearsed on a one-GPU box (both ranks on cuda:0, gloo collectives)
      # through bench.py's own launcher (`--gpus 2` without torch.distributed.run starts the ranks)
      DROID_BENCH_ONE_DEVICE=1 DROID_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 \
        --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_2rank.json" 2> "$O/bench_2rank.err" \
        || fail "$step" $? "$O/bench_2rank.err"
      cat "$O/bench_2rank.json" ;;
    rccl1)
      # the sharded path on RCCL with one rank (nccl backend initialised, device all-reduce of the
      # reduced system's tiles): the one-GPU box's check of what the 8-GPU node runs
      DROID_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 1 --config C3 --steps 3 --warmup 1 \
        --no-cpu-baseline > "$O/bench_rccl1.json" 2> "$O/bench_rccl1.err" || fail "$step" $? "$O/bench_rccl1.err"
      cat "$O/bench_rccl1.json" ;;
    env:*)
      # export K=V for the steps that follow (A/B runs: env:DROID_OVERLAP_GLO=0 bench:C3)
      export "${step#env:}"; echo "export ${step#env:}" ;;
    py:*)
      PYN=$((PYN+1)); PO="$O/py$PYN.txt"
      timeout -k 10 600 python -u ${step#py:} > "$PO" 2>&1 || fail "$step" $? "$PO"
      tail -30 "$PO" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
