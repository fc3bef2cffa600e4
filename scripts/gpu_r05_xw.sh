#!/bin/bash
# round 5: the exchange-wave split instance (pt_split_xw_kernel): split parity tests, stamps, C3/C5 timing with and
# without it (PQD_SPLIT_XW=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/${TAG:-xw}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robustness.py tests/test_gpu_branching.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -x -k "split or config3 or single or trunk or tomog" > $O/pytest_xw.log 2>&1
rc=$?
tail -4 $O/pytest_xw.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
timeout -k 10 200 python3 -u scripts/split_stamps.py --n-tau 2000 > $O/stamps_xw.log 2>&1 || exit 1
tail -24 $O/stamps_xw.log
for r in 1 2; do
  for xw in 1 0; do
    PQD_SPLIT_XW=$xw timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one,c3eight,c2one --steps 3 > $O/c3_xw$xw.$r.log 2>&1 || exit 1
    echo "xw=$xw"; grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*' $O/c3_xw$xw.$r.log | paste - -
  done
done
exit 0
