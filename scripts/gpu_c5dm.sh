#!/bin/bash
# C5 tomography scan at one rank's SURVEY share (32 points), its host/GPU split (cProfile) and kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/c5dm; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u scripts/bench_configs.py --configs c5dm32 --steps 1 > $O/c5dm32.log 2>&1 || { tail $O/c5dm32.log; exit 1; }
grep -o '"wall_s_per_scan": [0-9.]*\|"points_per_s": [0-9.]*' $O/c5dm32.log
timeout -k 10 300 python -u scripts/prof_c5dm.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep "profiled scan" $O/prof.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_configs.py --configs c5dm --steps 1 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/c5dm_kernel_stats.csv
