set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03bv; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --reference-layout --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_refl.json 2> $O/bench_refl.err || exit 1
ks=$(find $O/prof -name '*kernel_stats.csv' | head -n 1)
python3 $R/scripts/kstats.py $O/bench_refl.json $ks > $O/rocprof_top_refl.txt
head -25 $O/rocprof_top_refl.txt
