#!/bin/bash
# round 6: z|r in-kernel clock at C3 and C2 sizes (profiling build, after >= 2.5 s of back-to-back
# launches on random data), and the A/B bound on the z|r h re-read (DROID_ZR_NO_H)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O=gpurun_out/r06g
mkdir -p $O
export PYTHONUNBUFFERED=1
for E in 2048 96; do
  TL_WARM_S=2.5 TL_TILE=0 timeout -k 10 120 python -u scripts/conv_timeline.py $E zrp > $O/zrp_clock_$E.txt 2>&1 || { cat $O/zrp_clock_$E.txt; exit 1; }
  grep -E "zrp:|clock" $O/zrp_clock_$E.txt
done
timeout -k 10 120 python -u scripts/zr_nohb.py > $O/zr_no_h_ab.txt 2>&1 || { cat $O/zr_no_h_ab.txt; exit 1; }
cat $O/zr_no_h_ab.txt
