#!/bin/bash
# precomputed slice sums (PQD_PTSUM): parity under PTSUM=1, then the headline and c5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ptsum; mkdir -p $O
export TMPDIR=/tmp
PQD_PTSUM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_c5.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
timeout -k 10 400 python -u scripts/profile_sweep.py --n-tau 2000 --traj 2048 --pt-modes 4 --variants 0 --rounds 3 --env "PQD_PTSUM=0;PQD_PTSUM=1" > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
grep sweep $O/head.log
timeout -k 10 400 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0 --rounds 3 --env "PQD_PTSUM=0;PQD_PTSUM=1" > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
grep sweep $O/c5.log
