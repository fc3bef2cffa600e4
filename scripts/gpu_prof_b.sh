#!/bin/bash
# map-chain kernel summary + phase ablations of the C5 (six-level) and C2 (TLS quad) sweeps
set -o pipefail
O=gpurun_out/prof_b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mc -o mc --output-format csv -- python -u scripts/bench_mapchain.py --cases onetime --no-cpu > $O/mc.log 2>&1 || { echo "rocprof failed"; tail $O/mc.log; exit 1; }
find $O/mc -name "*kernel_stats.csv" -exec cp {} $O/mc_kernel_stats.csv \;
cut -d, -f1-4 $O/mc_kernel_stats.csv | head -20
grep case $O/mc.log
timeout -k 10 300 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 4 --variants 0,1,2,4,3 --rounds 2 > $O/abl_c5.log 2>&1 || { echo "c5 ablation failed"; tail $O/abl_c5.log; exit 1; }
grep sweep $O/abl_c5.log
timeout -k 10 300 python -u scripts/profile_sweep.py --config c2 --n-tau 4000 --pt-modes 4 --variants 0,1,2,4,3 --rounds 2 > $O/abl_c2.log 2>&1 || { echo "c2 ablation failed"; tail $O/abl_c2.log; exit 1; }
grep sweep $O/abl_c2.log
