#!/bin/bash
# round 6: timing-only ablations of the multi-trajectory split kernel (stamped instance; results not used)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-abl}
mkdir -p $O
for a in 0 128 384 0; do
  for t in 32 256; do
    timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 $t --ablate $a > $O/stamps_${t}_$a.log 2>&1 || exit 1
    grep -v Warning $O/stamps_${t}_$a.log | grep -v check
  done
done
exit 0
