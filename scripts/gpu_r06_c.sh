#!/bin/bash
# round 6: msplit vs batched over the t1 count, stamps of the current build, 8/20-run biexciton scans
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-c}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs c4ntraj --steps 2 > $O/c4ntraj.log 2>&1 || exit 1
grep -v Warn $O/c4ntraj.log | grep -v "check(" | cut -c1-400
for t in 32 256; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t > $O/stamps_$t.log 2>&1 || exit 1
  grep -v Warn $O/stamps_$t.log | grep -v "check("
done
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3eight,c3twenty,c5eight,c3one,c5one --steps 3 > $O/cfg.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"path": "[a-z ,-]*"\|"pt_sweep_ms": [0-9.]*' $O/cfg.log | paste - - -
exit 0
