#!/bin/bash
# quad kernel 4-column strips (PQD_QCG=1, four waves per SIMD) vs the default 8-column strips, C2
set -o pipefail
O=gpurun_out/quad_ab2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
for r in 1 2; do
  for q in 2 1; do
    PQD_QCG=$q timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q$q.log 2>&1 || { tail $O/q$q.log; exit 1; }
    echo "round $r qcg=$q: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q$q.log | tr '\n' ' ')"
  done
done
