#!/bin/bash
# quad kernel wave priorities (PQD_QPRIO 0..3), C2
set -o pipefail
O=gpurun_out/quad_prio
mkdir -p $O
export TMPDIR=/tmp
for q in 1 2 3; do
  PQD_QPRIO=$q timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest$q.log 2>&1; rc=$?
  echo "prio $q: $(tail -1 $O/pytest$q.log)"
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|Error" $O/pytest$q.log | head; exit 1; }
done
for r in 1 2; do
  for q in 0 1 2 3; do
    PQD_QPRIO=$q timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q$q.log 2>&1 || { tail $O/q$q.log; exit 1; }
    echo "round $r prio=$q: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q$q.log | tr '\n' ' ')"
  done
done
