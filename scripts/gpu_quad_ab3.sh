#!/bin/bash
# quad kernel: tree (dynamic priority, scalar fast-run bound, column MFMAs first) vs + ds_bpermute relayout, C2
set -o pipefail
O=gpurun_out/quad_ab3
mkdir -p $O
export TMPDIR=/tmp
for L in pyaceqd_amd/libpqd.so ab/libpqd_bperm.so; do
  PQD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
  echo "$L: $(tail -1 $O/pytest.log)"
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
done
for r in 1 2; do
  for L in pyaceqd_amd/libpqd.so ab/libpqd_bperm.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2,c2one --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
timeout -k 10 100 python -u scripts/quad_stamps.py --config c2 > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
cat $O/stamps.log
