#!/bin/bash
# final tree (rounds 5, 6): the other configs' bench lines (C2 frontend window, C4 stereo,
# update_lowmem, the 2-rank gloo rehearsal on one GPU, the sharded path on RCCL
# with one rank, the reference-API drop-in, C5) - each under its own time limit
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/${CFG_OUT:-r05cfg}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], round(d['value'], 3), round(d['ms_per_step'], 3))" $O/bench_$n.json $n
}
if [ "${CFG_SKIP_DONE:-0}" != 1 ]; then
run C2 python -u bench.py --config C2 --no-cpu-baseline
run C4 python -u bench.py --config C4 --no-cpu-baseline
run lowmem python -u bench.py --lowmem --no-cpu-baseline
run 2rank env DROID_BENCH_ONE_DEVICE=1 DROID_BENCH_BACKEND=gloo python -u bench.py --gpus 2 --no-cpu-baseline
fi
run rccl1 env DROID_BENCH_FORCE_DIST=1 python -u bench.py --no-cpu-baseline
run refapi python -u bench.py --reference-api --no-cpu-baseline
run C5 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline
