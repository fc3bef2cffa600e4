#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx05 --steps 20 --stats > $T/stats_bx05.log 2>&1 || { tail -20 $T/stats_bx05.log; exit 1; }
grep -E "STATS|RESULT" $T/stats_bx05.log
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/stats_bx01.log 2>&1 || { tail -20 $T/stats_bx01.log; exit 1; }
grep -E "STATS|RESULT" $T/stats_bx01.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx01 --steps 25 > $T/bench_ptgen_prof.log 2>&1 || { tail -30 $T/bench_ptgen_prof.log; exit 1; }
find /tmp/prof_ptgen -name "*kernel_stats*" -exec cp {} $T/ptgen_bx01_kernel_stats.csv \;
head -12 $T/ptgen_bx01_kernel_stats.csv
