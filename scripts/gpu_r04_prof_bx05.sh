#!/bin/bash
# kernel statistics of the biexciton default generator (K = 41, whole PT) and its phase split
set -o pipefail
mkdir -p gpurun_out/r04
T=gpurun_out/r04
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bx05 -o ptg -- python3 scripts/bench_ptgen.py --case bx05 > $T/prof_bx05.log 2>&1 || { tail -30 $T/prof_bx05.log; exit 1; }
find /tmp/prof_bx05 -name "*kernel_stats*" -exec cp {} $T/bx05_kernel_stats.csv \;
PQD_PTG_PHASES=1 timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx05 > $T/phases_bx05.log 2>&1 || { tail -20 $T/phases_bx05.log; exit 1; }
grep -E "PHASES|RESULT" $T/phases_bx05.log
