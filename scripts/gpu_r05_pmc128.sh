#!/bin/bash
# round 5: SQ counter passes of the chi = 128 dictionary sweep (c4d128s), the chi = 128 generated-PT oracle test and
# the use_infinite memory test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/pmc128
mkdir -p $O
export TMPDIR=/tmp
ARGS="--configs c4d128s --steps 1"
pass() { local name=$1; shift; echo "== $name"; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- python3 scripts/bench_configs.py $ARGS > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$name.log; exit 1; }; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ptgen.py -m gpu -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "chi128 or infinite_memory" > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
case $rc in 0|1) ;; *) echo "rc=$rc: stopping"; exit 1;; esac
pass sqA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
pass sqB SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
pass sqC SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE
exit $rc
