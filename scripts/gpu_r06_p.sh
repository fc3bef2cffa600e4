#!/bin/bash
# round 6: msplit tests, the t1 sweep, the C3/C5 small-batch rows, and a rocprofv3 kernel trace of the C4 rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-p}
mkdir -p $O
R=$(pwd)
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msplit.py > $O/pytest_msplit.log 2>&1 || { tail -30 $O/pytest_msplit.log; exit 1; }
tail -1 $O/pytest_msplit.log
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs c4ntraj --steps 2 > $O/c4ntraj.log 2>&1 || exit 1
grep -v Warn $O/c4ntraj.log | grep -v "check(" | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{\"n_traj'):
        d = json.loads(l); print(d['n_traj'], {k: (d[k]['path'][:12], d[k]['bt'], round(d[k]['us_per_step'], 2)) for k in ('msplit', 'auto', 'batched')})
"
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs c3eight,c3twenty,c5eight,c3one,c5one,c3one128 --steps 3 > $O/cfg.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"path": "[a-z ,-]*"\|"pt_sweep_ms": [0-9.]*' $O/cfg.log | paste - - -
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c4_trace -o c4 -- python3 -u $R/scripts/bench_configs.py --configs c4shard,c4full --steps 2 > $R/$O/c4_prof.log 2>&1 || exit 1
cd $R
grep -o '"config": "[a-z0-9]*"\|"sweep_ms": [0-9.]*' $O/c4_prof.log | paste - - - - -
find $O/c4_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -6 {}'
exit 0
