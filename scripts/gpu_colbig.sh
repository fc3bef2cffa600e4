#!/bin/bash
# N2 > 16 column phases (PQD_COLBIG): parity of the six-level / N = 5 paths, then the c5 sweep A/B and ablations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/colbig; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_c5.py tests/test_gpu_configs.py -k "not config2 and not config1" -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
timeout -k 10 400 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0,1,2,4 --rounds 3 --env "PQD_COLBIG=0;PQD_COLBIG=1" > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
grep sweep $O/c5.log
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"pt_sweep": [0-9.]*\|"frac": [0-9.]*' $O/bench.log | tr '\n' ' '
