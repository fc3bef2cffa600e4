#!/bin/bash
# round 4: where the headline kernel's non-MFMA cycles go. Three SQ counter passes (<= 8 SQ + 2 GRBM each, no trace
# domains combined with --pmc) over one full-size bench launch (n_tau = 10,000, 2,048 trajectories)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r04/pmc
export TMPDIR=/tmp
O=gpurun_out/r04/pmc
ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
pass() { local name=$1; shift; echo "== $name"; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- python3 bench.py $ARGS > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$name.log; exit 1; }; }
pass sqA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
pass sqB SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
pass sqC SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE
find $O -name "*counter_collection*.csv" | head
