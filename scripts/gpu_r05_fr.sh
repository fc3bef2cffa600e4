#!/bin/bash
# round 5: fused readout (PQD_FR=1): parity with it forced, then alternating bench runs; then the split stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/fr
mkdir -p $O gpurun_out/r05/split
export TMPDIR=/tmp
PQD_FR=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_windows.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -x > $O/pytest_fr1.log 2>&1
rc=$?
tail -4 $O/pytest_fr1.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
VARIANTS="PQD_FR=0
PQD_FR=1
PQD_FR=0
PQD_FR=1
PQD_FR=0
PQD_FR=1" bash scripts/gpu_ab.sh 2>&1 | tee $O/ab.log
timeout -k 10 200 python3 -u scripts/split_stamps.py --n-tau 2000 > gpurun_out/r05/split/stamps.log 2>&1
tail -22 gpurun_out/r05/split/stamps.log
exit 0
