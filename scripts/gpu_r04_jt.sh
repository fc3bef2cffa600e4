#!/bin/bash
# Jacobi on R2 vs on R2^H (Drmac-Veselic's second preconditioning): sweeps, SVD parity, generator time
set -o pipefail
mkdir -p gpurun_out/r04
T=gpurun_out/r04
PQD_PTG_JT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "svd or influence" > $T/pytest_jt.log 2>&1 || { tail -30 $T/pytest_jt.log; exit 1; }
tail -2 $T/pytest_jt.log
for jt in 0 1; do
  PQD_PTG_JT=$jt timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/jt_$jt.log 2>&1 || { tail -20 $T/jt_$jt.log; exit 1; }
  echo "JT $jt"; grep -oE "jacobi \(n, sweeps\): [^;]*|RESULT.*" $T/jt_$jt.log
done
