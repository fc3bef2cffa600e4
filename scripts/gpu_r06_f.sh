#!/bin/bash
# round 6: PT row values by DPP row broadcast (msplit) — tests, stamps (4096 = the broadcast-read PT), C4 rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-f}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msplit.py > $O/pytest_msplit.log 2>&1 || { tail -30 $O/pytest_msplit.log; exit 1; }
tail -3 $O/pytest_msplit.log
for t in 32 256; do for a in 0 4096; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t --ablate $a > $O/stamps_${t}_a$a.log 2>&1 || exit 1
  echo "== $t ablate $a"; grep -v Warn $O/stamps_${t}_a$a.log | grep -v "check(" | tail -12
done; done
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c4shard,c4full,c3one128 --steps 3 > $O/c4.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"sweep_ms": [0-9.]*' $O/c4.log | paste - - - - -
exit 0
