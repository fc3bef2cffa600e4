#!/bin/bash
# one GPU call: host<->device copy paths, the map-chain bench vs the reference Fortran, and its rocprofv3 kernel summary
# usage: scripts/gpu_mapchain.sh <tag>
set -o pipefail
T=${1:-mc}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/ubench_h2d.py > $O/ubench_h2d.log 2>&1 || { echo "ubench failed"; tail $O/ubench_h2d.log; exit 1; }
cat $O/ubench_h2d.log
timeout -k 10 600 python -u scripts/bench_mapchain.py --cases onetime,block,ft8 > $O/bench_mapchain.log 2>&1 || { echo "bench failed"; tail $O/bench_mapchain.log; exit 1; }
cat $O/bench_mapchain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o mc -- python -u scripts/bench_mapchain.py --cases onetime --no-cpu > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -20
