#!/bin/bash
# round 6: multi-trajectory split groups (pt_msplit.hip): parity tests, then the literal C4 rows (c4shard, c4full)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-ms}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msplit.py -m gpu -v \
    --timeout 300 --timeout-method thread -p no:cacheprovider -x ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_msplit.log 2>&1
rc=$?
tail -15 $O/pytest_msplit.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 32 > $O/stamps32.log 2>&1 || exit 1
cat $O/stamps32.log
timeout -k 10 120 python3 -u scripts/msplit_stamps.py --n-t1 256 > $O/stamps256.log 2>&1 || exit 1
cat $O/stamps256.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python3 -u scripts/bench_configs.py --configs ${CONFIGS:-c4shard,c4full} --steps 3 > $O/c4_rows.log 2>&1 || exit 1
cat $O/c4_rows.log
exit 0
