#!/bin/bash
# map-chain host-side phases: PQD_MC_TIMING on the bench's own cases and on the standalone breakdown
set -o pipefail
O=gpurun_out/mc_h
mkdir -p $O
export TMPDIR=/tmp
PQD_MC_TIMING=1 timeout -k 10 200 python -u scripts/bench_mapchain.py --cases onetime,block --no-cpu > $O/bench_t.log 2>&1 || { tail $O/bench_t.log; exit 1; }
grep -v Progress $O/bench_t.log | cut -c1-200
for d in 2 4 6; do
  timeout -k 10 100 python -u scripts/mc_breakdown.py --dim $d --reps 6 > $O/bd_$d.log 2>&1 || { tail $O/bd_$d.log; exit 1; }
  echo "dim $d"; tail -5 $O/bd_$d.log
done
timeout -k 10 100 python -u scripts/ubench_h2d.py --mb 41 > $O/ub.log 2>&1 && cat $O/ub.log
