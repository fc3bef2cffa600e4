#!/bin/bash
# QR/Jacobi kernel round 2: parity tests, QR microbenchmark (plain vs blocked), generator timing + kernel profile
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "not biexciton_reference_default" > $T/pytest_wg3.log 2>&1 || { tail -30 $T/pytest_wg3.log; exit 1; }
tail -3 $T/pytest_wg3.log
QK_SHAPES=2955x636,1365x384,640x273,200x60 QK_KINDS=householder,blocked timeout -k 10 200 python -u scripts/bench_qr_kinds.py > $T/qr_kinds_wg3.log 2>&1 || { tail -20 $T/qr_kinds_wg3.log; exit 1; }
cat $T/qr_kinds_wg3.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bx01_wg3.log 2>&1 || { tail -20 $T/bx01_wg3.log; exit 1; }
grep -E "RESULT" $T/bx01_wg3.log
PQD_PTG_BLOCKED=1 timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bx01_wg3_blocked.log 2>&1 || { tail -20 $T/bx01_wg3_blocked.log; exit 1; }
grep -E "RESULT" $T/bx01_wg3_blocked.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bench_ptgen_prof_wg3.log 2>&1 || { tail -30 $T/bench_ptgen_prof_wg3.log; exit 1; }
find /tmp/prof_ptgen -name "*kernel_stats*" -exec cp {} $T/ptgen_bx01_kernel_stats_wg3.csv \;
echo done
