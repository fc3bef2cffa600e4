#!/bin/bash
# round 6: chi = 128 split groups with streamed slice rows (no spills) — chi 128/256 tests, the chi-128 single run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-t}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msplit.py -k "chi128 or chi256" > $O/pytest_chi.log 2>&1 || { tail -40 $O/pytest_chi.log; exit 1; }
tail -1 $O/pytest_chi.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -k "chi128" > $O/pytest_cfg128.log 2>&1 || { tail -40 $O/pytest_cfg128.log; exit 1; }
tail -1 $O/pytest_cfg128.log
for r in 1 2; do
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one128 --steps 3 > $O/cfg_$r.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"path": "[a-z ,-]*"\|"pt_sweep_ms": [0-9.]*' $O/cfg_$r.log | paste - - -
done
exit 0
