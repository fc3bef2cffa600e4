#!/bin/bash
# PT unit lists in LDS + the slice schedule read at the top of the step: parity, then alternating builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ldsu; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
LIB_B=ab/libpqd_base.so ROUNDS=3 bash scripts/gpu_bench_lib_ab.sh || exit 1
for r in 1 2; do
  for lib in "" ab/libpqd_base.so; do
    PQD_LIB=$lib timeout -k 10 300 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0 --rounds 2 > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
    echo "[${lib:-current}] $(grep sweep $O/c5.log)"
  done
done
