#!/bin/bash
# round 5: the register-resident small QR (qr_reg_kernel): generator tests, then bx01 generator timing with and
# without it (PQD_PTG_QREG=0), shape statistics of a steady step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/${TAG:-qreg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ptgen.py -m gpu -q -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_ptgen.log 2>&1
rc=$?
tail -4 $O/pytest_ptgen.log
case $rc in 0) ;; *) echo "ptgen tests rc=$rc: stopping"; exit 1;; esac
for q in 1 0; do
  PQD_PTG_QREG=$q timeout -k 10 300 python3 -u scripts/bench_ptgen.py --case bx01,bx05 --steps ${STEPS:-60} > $O/bench_q$q.log 2>&1 || exit 1
  echo "qreg=$q"; grep RESULT $O/bench_q$q.log
done
exit 0
