#!/bin/bash
# quad kernel variants (ab/libpqd_q{a,b,c}.so vs the tree), C2
set -o pipefail
O=gpurun_out/quad_ab4
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for L in ab/libpqd_qh.so ab/libpqd_qt.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
