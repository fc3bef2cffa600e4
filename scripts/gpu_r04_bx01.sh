#!/bin/bash
# the biexciton default at dt = 0.1 (K = 205, threshold 1e-10): SVD scale tests, then the whole PT (410 steps +
# stationary slice), timed
set -o pipefail
mkdir -p gpurun_out/r04/full
T=gpurun_out/r04/full
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "svd or influence" > $T/pytest_svdscale.log 2>&1 || { tail -30 $T/pytest_svdscale.log; exit 1; }
tail -2 $T/pytest_svdscale.log
PQD_PTG_DUMP=$T/jacobi_fail.npy timeout -k 10 600 python -u scripts/bench_ptgen.py --case bx01 > $T/bench_ptgen_bx01_whole.log 2>&1 || { tail -30 $T/bench_ptgen_bx01_whole.log; exit 1; }
grep -E "RESULT|retries" $T/bench_ptgen_bx01_whole.log
