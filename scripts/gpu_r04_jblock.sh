#!/bin/bash
# block Jacobi: SVD / generator parity, then K = 205 timing (25 steps, with --stats for the sweep counts)
set -o pipefail
mkdir -p gpurun_out/r04/jb
T=gpurun_out/r04/jb
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "svd or influence or ibm or shift" > $T/pytest_jb.log 2>&1 || { tail -30 $T/pytest_jb.log; exit 1; }
tail -2 $T/pytest_jb.log
for jb in 1 0; do
  PQD_PTG_JBLOCK=$jb timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/jb_$jb.log 2>&1 || { tail -20 $T/jb_$jb.log; exit 1; }
  echo "JBLOCK $jb"; grep -oE "jacobi \(n, sweeps\): [^;]*|RESULT.*|retries.*" $T/jb_$jb.log
done
