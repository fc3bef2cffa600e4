#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptgen.py -x -v --timeout 300 --timeout-method thread -m gpu -k "timed or driver" \
    > gpurun_out/r04/pytest_ptgen_b.log 2>&1 || { tail -50 gpurun_out/r04/pytest_ptgen_b.log; exit 1; }
tail -3 gpurun_out/r04/pytest_ptgen_b.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 \
    --timeout-method thread -m gpu -k "rabi_kat or c1_vs_oracle or config1 or block_mode" \
    > gpurun_out/r04/pytest_touched.log 2>&1 || { tail -50 gpurun_out/r04/pytest_touched.log; exit 1; }
tail -3 gpurun_out/r04/pytest_touched.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx05 > gpurun_out/r04/bench_ptgen_prof.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen_prof.log; exit 1; }
grep RESULT gpurun_out/r04/bench_ptgen_prof.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case tls > gpurun_out/r04/bench_ptgen_tls.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen_tls.log; exit 1; }
grep RESULT gpurun_out/r04/bench_ptgen_tls.log
timeout -k 10 400 python -u scripts/bench_ptgen.py --case bx01 --steps 41 > gpurun_out/r04/bench_ptgen_bx01.log 2>&1 || { tail -30 gpurun_out/r04/bench_ptgen_bx01.log; exit 1; }
grep RESULT gpurun_out/r04/bench_ptgen_bx01.log
