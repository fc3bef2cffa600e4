#!/bin/bash
# matrix-core free propagators at N2 = 16 (PQD_FPM=2): parity, then the headline bench A/B (free_prop kernel ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/fpm16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "free_prop" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_fp.log 2>&1
rc=$?; tail -3 $O/pytest_fp.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest_fp.log | head; echo "rc=$rc stop"; exit 1;; esac
for f in 1 2 1 2 1 2; do
  PQD_FPM=$f timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$f.log 2>&1 || { tail $O/bench_$f.log; exit 1; }
  echo "FPM=$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"free_prop": [0-9.]*' $O/bench_$f.log | tr '\n' ' ')"
done
for f in 1 2; do
  PQD_FPM=$f timeout -k 10 300 python -u scripts/bench_configs.py --configs c3one > $O/c3one_$f.log 2>&1 || { tail $O/c3one_$f.log; exit 1; }
  echo "FPM=$f c3one $(grep -o '"wall_ms[a-z_]*": [0-9.]*\|"free_prop_ms": [0-9.]*' $O/c3one_$f.log | tr '\n' ' ')"
done
