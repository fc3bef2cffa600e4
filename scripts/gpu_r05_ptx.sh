#!/bin/bash
# round 5: PQD_PTX variants of the headline PT unit loop: parity (test_gpu_parity.py with the variant forced), then
# alternating bench runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/ptx
mkdir -p $O
export TMPDIR=/tmp
PQD_PTX=7 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py -m gpu -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -x > $O/pytest_ptx7.log 2>&1
rc=$?
tail -4 $O/pytest_ptx7.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
VARIANTS="PQD_PTX=0
PQD_PTX=2
PQD_PTX=3
PQD_PTX=6
PQD_PTX=7
PQD_PTX=1
PQD_PTX=0
PQD_PTX=7
PQD_PTX=6
PQD_PTX=3
PQD_PTX=2" bash scripts/gpu_ab.sh 2>&1 | tee $O/ab.log
exit 0
