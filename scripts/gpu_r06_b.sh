#!/bin/bash
# round 6: chi = 128 split groups (tests + the c3one128 row, with and without), the C4 rows under rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msplit.py tests/test_gpu_parity.py -m gpu -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "msplit or sweep_pt" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log
case $rc in 0) ;; *) echo "tests rc=$rc: stopping"; exit 1;; esac
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one128,c3one --steps 3 > $O/c3one128.log 2>&1 || exit 1
PQD_MSPLIT=0 timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one128 --steps 3 > $O/c3one128_batched.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"path": "[a-z ,-]*"\|"pt_sweep_ms": [0-9.]*' $O/c3one128.log $O/c3one128_batched.log | paste - - -
[ -n "$NO_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 -- python3 -u scripts/bench_configs.py --configs c4shard,c4full --steps 2 > $O/c4_prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -3
exit 0
