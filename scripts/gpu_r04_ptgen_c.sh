#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_ptgen.py -x -v --timeout 300 --timeout-method thread -m gpu \
    > gpurun_out/r04/pytest_ptgen.log 2>&1 || { tail -50 gpurun_out/r04/pytest_ptgen.log; exit 1; }
tail -3 gpurun_out/r04/pytest_ptgen.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_correlations_golden.py -x -v --timeout 200 \
    --timeout-method thread -m gpu -k "map_tail or phonon_map" > gpurun_out/r04/pytest_maptail.log 2>&1 || { tail -50 gpurun_out/r04/pytest_maptail.log; exit 1; }
tail -3 gpurun_out/r04/pytest_maptail.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx05 --steps 20 > gpurun_out/r04/bench_ptgen_prof.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen_prof.log; exit 1; }
find /tmp/prof_ptgen | head -20
find /tmp/prof_ptgen -name "*stats*" -exec cp {} gpurun_out/r04/ \;
timeout -k 10 300 python3 -m cProfile -s tottime scripts/bench_ptgen.py --case bx05 --steps 20 > gpurun_out/r04/cprof_ptgen.log 2>&1 || { tail -30 gpurun_out/r04/cprof_ptgen.log; exit 1; }
head -30 gpurun_out/r04/cprof_ptgen.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx05,tls > gpurun_out/r04/bench_ptgen.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen.log; exit 1; }
grep RESULT gpurun_out/r04/bench_ptgen.log
timeout -k 10 400 python -u scripts/bench_ptgen.py --case bx01 --steps 60 > gpurun_out/r04/bench_ptgen_bx01.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen_bx01.log; exit 1; }
grep RESULT gpurun_out/r04/bench_ptgen_bx01.log
