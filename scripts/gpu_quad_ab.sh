#!/bin/bash
# quad kernel: parity tests, then alternating A/B of C2 (bench_configs c2) between ab/libpqd_base.so and the tree's build
set -o pipefail
O=gpurun_out/quad_ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_configs.py -k "quad or config2" -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
for r in 1 2 3; do
  PQD_LIB=ab/libpqd_base.so timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/base_$r.log 2>&1 || { tail $O/base_$r.log; exit 1; }
  timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/new_$r.log 2>&1 || { tail $O/new_$r.log; exit 1; }
  echo "round $r: base $(grep -o '"pt_sweep_ms": [0-9.]*' $O/base_$r.log) frac $(grep -o '"frac_fp64": [0-9.]*' $O/base_$r.log) | new $(grep -o '"pt_sweep_ms": [0-9.]*' $O/new_$r.log) frac $(grep -o '"frac_fp64": [0-9.]*' $O/new_$r.log)"
done
