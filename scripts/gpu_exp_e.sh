#!/bin/bash
set -o pipefail
O=gpurun_out/exp_e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "contraction_modes or config_workloads or sweep_pt or multi_system or branching" tests/test_gpu_branching.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
for v in "PQD_COL44=0 PQD_PT_MODE=4" "PQD_COL44=1 PQD_PT_MODE=4" "PQD_COL44=0 PQD_PT_MODE=5" "PQD_COL44=1 PQD_PT_MODE=5" "PQD_COL44=1 PQD_PT_MODE=6"; do
  env $v timeout -k 10 200 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes ${v##*=} --variants 0 --rounds 3 > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
  echo "$v: $(grep sweep $O/c5.log)"
done
