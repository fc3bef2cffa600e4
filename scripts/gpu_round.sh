#!/bin/bash
# one GPU call: the -m gpu suite, the bench line, and a rocprofv3 kernel summary of the map-chain bench
# usage: scripts/gpu_round.sh <tag>
set -o pipefail
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=40 \
    -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
