#!/bin/bash
# quad C2 instance: kept build (slow-step operator/event addresses via opq) vs v2 (+ activation source re-read) and
# v3 (+ event-list end re-read): quad tests on each, C2 in three alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/qv23; mkdir -p $O; export TMPDIR=/tmp
for L in abq/libpqd_v2.so abq/libpqd_v3.so; do
  PQD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
  echo "$L: $(tail -1 $O/pytest.log)"
done
for r in 1 2 3; do
  for L in pyaceqd_amd/libpqd.so abq/libpqd_v2.so abq/libpqd_v3.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
