#!/bin/bash
# matrix-core free propagators for N2 = 25, 36 (PQD_FPM): parity, then the C5 configs A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/fpm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "free_prop" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_fp.log 2>&1
rc=$?; tail -3 $O/pytest_fp.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest_fp.log | head; echo "rc=$rc stop"; exit 1;; esac
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py tests/test_gpu_configs.py -k "not config2 and not config1 and not config3" -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for f in 1 2 1 2; do
  PQD_FPM=$f timeout -k 10 300 python -u scripts/bench_configs.py --configs c5 > $O/c5_$f.log 2>&1 || { tail $O/c5_$f.log; exit 1; }
  echo "FPM=$f $(grep -o '"wall_ms_per_launch": [0-9.]*\|"free_prop_ms": [0-9.]*' $O/c5_$f.log | tr '\n' ' ')"
done
PQD_FPM=2 timeout -k 10 300 python -u scripts/bench_configs.py --configs c5dm > $O/c5dm.log 2>&1 || { tail $O/c5dm.log; exit 1; }
grep -o '"wall_s_per_scan": [0-9.]*' $O/c5dm.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PQD_FPM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_configs.py --configs c5 --steps 1 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/c5_kernel_stats.csv
