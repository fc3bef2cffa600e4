#!/bin/bash
# wave-per-output traces at N2 > 16 (PQD_TRPRE=0 selects the per-output loop): parity, then C5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/wavetr; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_c5.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
timeout -k 10 400 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0,4 --rounds 3 --env "PQD_TRPRE=0;PQD_TRPRE=1" > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
grep sweep $O/c5.log
for u in 0 1; do
  PQD_TRPRE=$u timeout -k 10 300 python -u scripts/bench_configs.py --configs c5,c5d,c5dm --steps 2 > $O/cfg_$u.log 2>&1 || { tail $O/cfg_$u.log; exit 1; }
  echo "TRPRE=$u $(grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*\|"wall_s_per_scan": [0-9.]*' $O/cfg_$u.log | tr '\n' ' ')"
done
