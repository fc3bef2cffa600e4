#!/bin/bash
# round 6: chi = 256 on multi-trajectory split groups (streamed slice rows) and the uncapped-bond IBM test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-q}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_msplit.py -k "chi256 or chi128" > $O/pytest_chi256.log 2>&1 || { tail -40 $O/pytest_chi256.log; exit 1; }
tail -3 $O/pytest_chi256.log
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_ptgen.py -k "uncapped" --durations=3 > $O/pytest_uncapped.log 2>&1 || { tail -40 $O/pytest_uncapped.log; exit 1; }
grep -E "tls 1e-10|passed|failed" $O/pytest_uncapped.log | tail -5
exit 0
