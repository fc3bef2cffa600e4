#!/bin/bash
# round 6: per-wave gather timing of the multi-trajectory split groups (stamped build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-h}
mkdir -p $O
for t in ${NT1:-256 32}; do for a in ${ABL:-0}; do
  timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t --ablate $a > $O/stamps_${t}_a$a.log 2>&1 || exit 1
  echo "== $t ablate $a"; grep -v Warn $O/stamps_${t}_a$a.log | grep -v "check(" | tail -28
done; done
exit 0
