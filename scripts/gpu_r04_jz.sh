#!/bin/bash
# Jacobi sweeps vs the zero-column threshold (boundary SVDs of the K = 205 biexciton generator)
set -o pipefail
mkdir -p gpurun_out/r04
T=gpurun_out/r04
for z in 1e-16 1e-15 1e-14; do
  PQD_PTG_JZERO=$z timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/jz_$z.log 2>&1 || { tail -20 $T/jz_$z.log; exit 1; }
  echo "zero_tol $z"; grep -oE "jacobi \(n, sweeps\): [^;]*|RESULT.*" $T/jz_$z.log
done
