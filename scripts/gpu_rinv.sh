#!/bin/bash
# Horner steps of the matrix-core free-propagator builders multiply by 1/mm from a constant table (ab/libpqd_rinv.so)
# instead of dividing (ab/libpqd_fp4m.so); libpqd.so adds the register-resident N2 = 4 fuse kernel: parity, then
# C1 / C2 / C5 A/B in alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/rinv; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_robustness.py tests/test_gpu_c5.py tests/test_gpu_quad.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_fp4m.so ab/libpqd_rinv.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 200 python scripts/bench_configs.py --configs c1,c2,c5 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"config": "[a-z0-9]*"\|"wall_ms_per_launch": [0-9.]*\|"free_prop_ms": [0-9.]*' $O/q.log | tr '\n' ' ')" | tee -a $O/ab.log
  done
done
