#!/bin/bash
# workgroup-per-column step kernels + blocked Q formation: parity tests, QR microbenchmark, generator timing
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptgen.py -k "not biexciton_reference_default" > $T/pytest_wg.log 2>&1 || { tail -30 $T/pytest_wg.log; exit 1; }
tail -3 $T/pytest_wg.log
QK_SHAPES=2955x636,1365x384,640x273,200x60 timeout -k 10 200 python -u scripts/bench_qr_kinds.py > $T/qr_kinds_wg.log 2>&1 || { tail -20 $T/qr_kinds_wg.log; exit 1; }
cat $T/qr_kinds_wg.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/stats_bx01_wg.log 2>&1 || { tail -20 $T/stats_bx01_wg.log; exit 1; }
grep -E "STATS|RESULT" $T/stats_bx01_wg.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bench_ptgen_prof_wg.log 2>&1 || { tail -30 $T/bench_ptgen_prof_wg.log; exit 1; }
find /tmp/prof_ptgen -name "*kernel_stats*" -exec cp {} $T/ptgen_bx01_kernel_stats_wg.csv \;
cut -c1-150 $T/ptgen_bx01_kernel_stats_wg.csv | head -14
