#!/bin/bash
set -o pipefail
O=gpurun_out/exp_c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python scripts/ubench_h2d.py --mb 42 > $O/ubench.log 2>&1 || { echo ubench failed; tail $O/ubench.log; exit 1; }
cat $O/ubench.log
timeout -k 10 300 python -u scripts/bench_mapchain.py --cases onetime > $O/mc.log 2>&1 || { echo mc failed; tail $O/mc.log; exit 1; }
grep case $O/mc.log
timeout -k 10 300 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 4,5 --variants 0 --rounds 3 > $O/c5_ptmode.log 2>&1 || { echo c5 failed; tail $O/c5_ptmode.log; exit 1; }
grep sweep $O/c5_ptmode.log
