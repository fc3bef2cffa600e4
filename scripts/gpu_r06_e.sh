#!/bin/bash
# round 6: what the gather of 8 trajectories per workgroup waits for (stamped build variants, timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-e}
mkdir -p $O
for a in 0 1024 2048 1152; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 256 --ablate $a > $O/stamps_256_a$a.log 2>&1 || exit 1
  echo "== ablate $a"; grep -v Warn $O/stamps_256_a$a.log | grep -v "check(" | tail -10
done
exit 0
