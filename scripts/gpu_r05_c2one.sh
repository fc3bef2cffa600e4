#!/bin/bash
# round 5: the two-level single run (C2 shape, one trajectory) on split groups (PQD_SPLIT=2) vs the default path
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/c2one
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for sp in 1 2; do
    PQD_SPLIT=$sp timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c2one --steps 3 > $O/c2one_split$sp.$r.log 2>&1 || exit 1
    echo "PQD_SPLIT=$sp"; grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*' $O/c2one_split$sp.$r.log | paste - -
  done
done
exit 0
