#!/bin/bash
# block Jacobi (batched loads, register rotations): SVD / generator parity, then the biexciton default (K = 41, whole
# PT) and 25 steps of K = 205, block kernel vs the column-pair kernel
set -o pipefail
mkdir -p gpurun_out/r04/jb2
T=gpurun_out/r04/jb2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "svd or influence or ibm or shift" > $T/pytest_jb.log 2>&1 || { tail -30 $T/pytest_jb.log; exit 1; }
tail -2 $T/pytest_jb.log
for jb in 1 0; do
  PQD_PTG_JBLOCK=$jb timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx05 --stats > $T/bx05_jb$jb.log 2>&1 || { tail -20 $T/bx05_jb$jb.log; exit 1; }
  echo "JBLOCK $jb: $(grep -oE 'jacobi \(n, sweeps\): [^;]*' $T/bx05_jb$jb.log) $(grep -oE 'RESULT.*' $T/bx05_jb$jb.log)"
  PQD_PTG_JBLOCK=$jb timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/bx01_jb$jb.log 2>&1 || { tail -20 $T/bx01_jb$jb.log; exit 1; }
  echo "JBLOCK $jb: $(grep -oE 'jacobi \(n, sweeps\): [^;]*' $T/bx01_jb$jb.log) $(grep -oE 'RESULT.*' $T/bx01_jb$jb.log)"
done
