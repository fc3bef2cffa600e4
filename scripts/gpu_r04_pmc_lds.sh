#!/bin/bash
# round 4: which phase of the headline kernel makes its LDS bank conflicts: one SQ pass per PQD_ABLATE variant
# (0 full, 1 no PT contraction, 2 no column phases, 4 no outputs; outputs wrong by construction in 1/2/4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r04/pmc_lds
export TMPDIR=/tmp
O=gpurun_out/r04/pmc_lds
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --n-tau 2000"
for ab in 0 1 2 4; do
  echo "== ablate $ab"
  PQD_ABLATE=$ab timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/ab$ab -o run --output-format csv -- python3 bench.py $ARGS > $O/ab$ab.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/ab$ab.log; exit 1; }
done
