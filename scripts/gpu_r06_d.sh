#!/bin/bash
# round 6: exchange stores that keep their L2 lines (PQD_MS_L2) — msplit tests, C4 rows A/B, stamps, the t1 sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-d}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msplit.py > $O/pytest_msplit.log 2>&1 || { tail -30 $O/pytest_msplit.log; exit 1; }
tail -3 $O/pytest_msplit.log
for l2 in 0 1; do
  PQD_MS_L2=$l2 timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c4shard,c4full --steps 3 > $O/c4_l2$l2.log 2>&1 || exit 1
  grep -o '"config": "[a-z0-9]*"\|"sweep_ms": [0-9.]*' $O/c4_l2$l2.log | paste - - - - -
done
for t in 32 256; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t > $O/stamps_$t.log 2>&1 || exit 1
  grep -v Warn $O/stamps_$t.log | grep -v "check(" | tail -9
done
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs c4ntraj --steps 2 > $O/c4ntraj.log 2>&1 || exit 1
grep -v Warn $O/c4ntraj.log | grep -v "check(" | cut -c1-300
exit 0
