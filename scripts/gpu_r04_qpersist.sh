#!/bin/bash
# (1) quad kernel without scratch vs the round-4 head (ab/libpqd_base.so): quad/branching/CW tests, C2 A/B x3;
# (2) persistent QR: generator QR/SVD tests, then the biexciton generator with PQD_PTG_QPERSIST=0 / 1 (pivoted) / 2 (+plain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/qpersist; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_QUAD:-0}" = 0 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py "tests/test_gpu_configs.py::test_cw_drive_matches_exact_lindblad_solution" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_quad.log 2>&1
rc=$?; tail -2 $O/pytest_quad.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest_quad.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_base.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_ptgen.py -k "qr or svd" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_ptgen.log 2>&1
rc=$?; tail -2 $O/pytest_ptgen.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest_ptgen.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2; do
  for P in 0 1 2; do
    PQD_PTG_QPERSIST=$P PQD_PTG_PHASES=1 timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx05,bx01 --steps 25 > $O/ptg_$P.log 2>&1 || { tail -20 $O/ptg_$P.log; exit 1; }
    echo "round $r QPERSIST=$P: $(grep -E 'RESULT|PHASES' $O/ptg_$P.log | tr '\n' ' ')"
  done
done
