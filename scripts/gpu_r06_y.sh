#!/bin/bash
# round 6: narrow groups (one PT row per workgroup, two workgroups per CU) for small biexciton batches: tests, C4 shard A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-y}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msplit.py > $O/pytest_msplit.log 2>&1 || { tail -30 $O/pytest_msplit.log; exit 1; }
tail -1 $O/pytest_msplit.log
for r in 1 0 1 0; do
  PQD_MS_R1=$r timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c4shard --steps 3 > $O/c4shard_r1$r.log 2>&1 || exit 1
  echo "PQD_MS_R1=$r $(grep -o '"sweep_ms": [0-9.]*' $O/c4shard_r1$r.log | head -1)"
done
exit 0
