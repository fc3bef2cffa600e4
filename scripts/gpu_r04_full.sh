#!/bin/bash
# round 4 evidence: the whole -m gpu suite (one process), then whole-PT generator timings (K = 41, 64, 205)
set -o pipefail
mkdir -p gpurun_out/r04/full
export PYTHONUNBUFFERED=1
T=gpurun_out/r04/full
timeout -k 10 1500 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu --durations=25 > $T/pytest_gpu_all.log 2>&1 || { tail -60 $T/pytest_gpu_all.log; exit 1; }
tail -30 $T/pytest_gpu_all.log | grep -E "passed|failed|slowest|s call" | head -30
timeout -k 10 400 python -u scripts/bench_ptgen.py --case bx05,tls > $T/bench_ptgen_whole.log 2>&1 || { tail -30 $T/bench_ptgen_whole.log; exit 1; }
grep RESULT $T/bench_ptgen_whole.log
timeout -k 10 600 python -u scripts/bench_ptgen.py --case bx01 > $T/bench_ptgen_bx01_whole.log 2>&1 || { tail -30 $T/bench_ptgen_bx01_whole.log; exit 1; }
grep RESULT $T/bench_ptgen_bx01_whole.log
