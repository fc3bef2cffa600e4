#!/bin/bash
# round 6: single-trajectory split groups with the PT row values by DPP row broadcast — split tests, C3/C5 single rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-s}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_msplit.py -k "split or trunk" > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
for r in 1 2; do
timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one,c5one,c3eight --steps 3 > $O/cfg_$r.log 2>&1 || exit 1
grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*' $O/cfg_$r.log | paste - -
done
exit 0
