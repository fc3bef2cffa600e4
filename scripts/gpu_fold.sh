#!/bin/bash
# fold A/B: parity suites under PQD_FOLD=1 and 2, then bench variants alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/fold; mkdir -p $O
export TMPDIR=/tmp
for f in 1 2; do
  PQD_FOLD=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_fold$f.log 2>&1
  rc=$?; tail -3 $O/pytest_fold$f.log; case $rc in 0|1) ;; *) echo "rc=$rc stop"; exit 1;; esac
done
VARIANTS="PQD_FOLD=0
PQD_FOLD=1
PQD_FOLD=2
PQD_FOLD=0
PQD_FOLD=1
PQD_FOLD=2" BENCH_STEPS=4 bash scripts/gpu_ab.sh
