#!/bin/bash
# round 5: split groups with the output workgroup (G = N2 + 1): split parity tests, stamps with and without it,
# C3/C5 single-run timing with and without it (PQD_SPLIT_OW=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/${TAG:-ow}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robustness.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -x -k "split or config3 or single or trunk or tomog" > $O/pytest_ow.log 2>&1
rc=$?
tail -4 $O/pytest_ow.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
for ow in 1 0; do
  timeout -k 10 200 python3 -u scripts/split_stamps.py --n-tau 2000 --ow $ow > $O/stamps_ow$ow.log 2>&1 || exit 1
  tail -20 $O/stamps_ow$ow.log
done
for r in 1 2; do
  for ow in 1 0; do
    PQD_SPLIT_OW=$ow timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one,c5one,c3eight --steps 3 > $O/c3_ow$ow.$r.log 2>&1 || exit 1
    echo "ow=$ow"; grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*' $O/c3_ow$ow.$r.log | paste - -
  done
done
exit 0
