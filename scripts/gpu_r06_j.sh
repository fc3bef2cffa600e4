#!/bin/bash
# round 6: coalesced gather lanes in the multi-trajectory split groups — tests, stamps, C4 rows, the t1 sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-j}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msplit.py > $O/pytest_msplit.log 2>&1 || { tail -30 $O/pytest_msplit.log; exit 1; }
tail -2 $O/pytest_msplit.log
for t in 256 32; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t > $O/stamps_$t.log 2>&1 || exit 1
  echo "== $t"; grep -v Warn $O/stamps_$t.log | grep -v "check(" | tail -14
done
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c4shard,c4full,c3one128 --steps 3 > $O/c4.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"sweep_ms": [0-9.]*\|"pt_sweep_ms": [0-9.]*' $O/c4.log | paste - - - - -
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs c4ntraj --steps 2 > $O/c4ntraj.log 2>&1 || exit 1
grep -v Warn $O/c4ntraj.log | grep -v "check(" | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{\"n_traj'):
        d = json.loads(l); print(d['n_traj'], {k: (d[k]['path'][:12], d[k]['bt'], round(d[k]['us_per_step'], 2)) for k in ('msplit', 'auto', 'batched')})
"
exit 0
