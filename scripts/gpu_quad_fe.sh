#!/bin/bash
# quad kernel: fast-run end found once per entry (tree) vs two ballots per pair (ab/libpqd_base.so); parity, C2 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/quad_fe2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_base.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
