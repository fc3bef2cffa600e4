#!/bin/bash
# device trapezoid integrals for the tomography scan (PQD_SCAN_TRAPZ): parity, then c5dm A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/trapz; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "trapz or tables" tests/test_gpu_c5.py tests/test_gpu_configs.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "trapz or tables or c5 or config5" > $O/pytest.log 2>&1
rc=$?; tail -12 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for u in 0 1 0 1; do
  PQD_SCAN_TRAPZ=$u timeout -k 10 300 python -u scripts/bench_configs.py --configs c5dm --steps 2 > $O/c5dm_$u.log 2>&1 || { tail $O/c5dm_$u.log; exit 1; }
  echo "TRAPZ=$u $(grep -o '"wall_s_per_scan": [0-9.]*\|"concurrence": \[[0-9., e-]*' $O/c5dm_$u.log | tr '\n' ' ' | cut -c1-200)"
done
