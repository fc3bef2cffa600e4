#!/bin/bash
# blocked plain QR: parity tests, QR microbenchmark, generator timing at K = 205 (25 steps)
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "blocked or qr_matches or svd_matches" > $T/pytest_blocked.log 2>&1 || { tail -30 $T/pytest_blocked.log; exit 1; }
tail -3 $T/pytest_blocked.log
timeout -k 10 200 python -u scripts/bench_qr_kinds.py > $T/qr_kinds.log 2>&1 || { tail -20 $T/qr_kinds.log; exit 1; }
cat $T/qr_kinds.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/stats_bx01_blocked.log 2>&1 || { tail -20 $T/stats_bx01_blocked.log; exit 1; }
grep -E "STATS|RESULT" $T/stats_bx01_blocked.log
