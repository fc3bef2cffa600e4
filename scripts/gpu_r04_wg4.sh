#!/bin/bash
# QR/Jacobi kernel round 2: parity tests, QR microbenchmark (plain vs blocked), generator timing + kernel profile
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "not biexciton_reference_default" > $T/pytest_wg4.log 2>&1 || { tail -30 $T/pytest_wg4.log; exit 1; }
tail -3 $T/pytest_wg4.log
QK_SMALL=1 timeout -k 10 200 python -u scripts/bench_qr_kinds.py > $T/qr_kinds_wg4.log 2>&1 || { tail -20 $T/qr_kinds_wg4.log; exit 1; }
cat $T/qr_kinds_wg4.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bx01_wg4.log 2>&1 || { tail -20 $T/bx01_wg4.log; exit 1; }
grep -E "RESULT" $T/bx01_wg4.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bench_ptgen_prof_wg4.log 2>&1 || { tail -30 $T/bench_ptgen_prof_wg4.log; exit 1; }
find /tmp/prof_ptgen -name "*kernel_stats*" -exec cp {} $T/ptgen_bx01_kernel_stats_wg4.csv \;
echo done
