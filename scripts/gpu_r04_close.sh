#!/bin/bash
# closing check on the final head: quad/branching/config tests, then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r04d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py tests/test_gpu_configs.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_close.log 2>&1
rc=$?; tail -2 $O/pytest_close.log; case $rc in 0) ;; *) grep -E "^FAILED" $O/pytest_close.log | head; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/c2.log 2>&1 && grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/c2.log | tr '\n' ' '
