#!/bin/bash
# round 5: split-group output pass staged in LDS: split parity tests, stamps, C3 single-run timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/split
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robustness.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -x -k "split or config3 or single" > $O/pytest_split.log 2>&1
rc=$?
tail -4 $O/pytest_split.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
timeout -k 10 200 python3 -u scripts/split_stamps.py --n-tau 2000 > $O/stamps_${TAG:-after}.log 2>&1 || exit 1
tail -20 $O/stamps_${TAG:-after}.log
for r in 1 2; do
  timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one,c5one,c3eight --steps 3 > $O/c3one_${TAG:-after}.$r.log 2>&1 || exit 1
  grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*' $O/c3one_${TAG:-after}.$r.log | paste - - 
done
exit 0
