#!/bin/bash
# balanced PT row units (PQD_UNITBAL): parity, then the dictionary six-level configs A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/unitbal; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_c5.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
timeout -k 10 400 python -u scripts/profile_sweep.py --config c5d --n-tau 1000 --pt-modes 5 --variants 0 --rounds 3 --env "PQD_UNITBAL=0;PQD_UNITBAL=1" > $O/c5d.log 2>&1 || { tail $O/c5d.log; exit 1; }
grep sweep $O/c5d.log
timeout -k 10 400 python -u scripts/profile_sweep.py --config c3d --n-tau 2000 --pt-modes 4 --variants 0 --rounds 3 --env "PQD_UNITBAL=0;PQD_UNITBAL=1" > $O/c3d.log 2>&1 || { tail $O/c3d.log; exit 1; }
grep sweep $O/c3d.log
for u in 0 1; do
  PQD_UNITBAL=$u timeout -k 10 300 python -u scripts/bench_configs.py --configs c5dm --steps 2 > $O/c5dm_$u.log 2>&1 || { tail $O/c5dm_$u.log; exit 1; }
  echo "UNITBAL=$u $(grep -o '"wall_s_per_scan": [0-9.]*' $O/c5dm_$u.log)"
done
