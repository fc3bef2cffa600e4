#!/bin/bash
# boundary-SVD QRCP rank tolerance: Jacobi size and generator time at the biexciton default (K = 41), 25 steps of K = 205
set -o pipefail
mkdir -p gpurun_out/r04/rt
T=gpurun_out/r04/rt
for rt in 1e-14 1e-13 1e-12 1e-11; do
  PQD_PTG_RANKTOL=$rt timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx05 --steps 60 --stats > $T/bx05_$rt.log 2>&1 || { tail -20 $T/bx05_$rt.log; exit 1; }
  echo "ranktol $rt: $(grep -oE 'jacobi \(n, sweeps\): [^;]*' $T/bx05_$rt.log) $(grep -oE 'RESULT.*' $T/bx05_$rt.log)"
done
for rt in 1e-14 1e-12; do
  PQD_PTG_RANKTOL=$rt timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/bx01_$rt.log 2>&1 || { tail -20 $T/bx01_$rt.log; exit 1; }
  echo "ranktol $rt: $(grep -oE 'jacobi \(n, sweeps\): [^;]*' $T/bx01_$rt.log) $(grep -oE 'RESULT.*' $T/bx01_$rt.log)"
done
