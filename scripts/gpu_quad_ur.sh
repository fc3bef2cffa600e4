#!/bin/bash
# quad kernel: reload-free bodies without the schedule fetch (ab/libpqd_a.so) and additionally four steps per loop
# iteration (libpqd.so) vs the previous head (ab/libpqd_base.so); parity first, then C2 A/B in alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/quad_ur; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_base.so ab/libpqd_a.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')" | tee -a $O/ab_c2.log
  done
done
# where the C2 / C1 wall time goes outside the sweep (free propagators, windows, fusion)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o c2 --output-format csv -- python3 scripts/bench_configs.py --configs c2,c1 --steps 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
