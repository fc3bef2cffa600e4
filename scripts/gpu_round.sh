#!/bin/bash
# one GPU call: the BASELINE config tests, the whole -m gpu suite, the bench line
# usage: scripts/gpu_round.sh <tag> [nobench]
set -o pipefail
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 240 --timeout-method thread \
    --durations=10 -p no:cacheprovider > $O/pytest_configs.log 2>&1
rc=$?
tail -14 $O/pytest_configs.log
case $rc in 0|1) ;; *) echo "config tests rc=$rc: stopping"; exit 1;; esac
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40 \
    --deselect tests/test_gpu_configs.py -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc2=$?
tail -12 $O/pytest_gpu.log
case $rc2 in 0|1) ;; *) echo "suite rc=$rc2: stopping"; exit 1;; esac
[ "$2" = "nobench" ] && exit $((rc | rc2))
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
exit $((rc | rc2))
