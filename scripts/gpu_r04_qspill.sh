#!/bin/bash
# quad kernel without scratch (slow-step addresses re-derived in the slow step, pt_quad.hip opq) vs the round-4 head
# (ab/libpqd_base.so, 64 B scratch): parity (quad, branching, CW exact-solution tests), C2 A/B in three alternating
# rounds, one SQ counter pass on the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/qspill; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_branching.py "tests/test_gpu_configs.py::test_cw_drive_matches_exact_lindblad_solution" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_base.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d $GRAFT_REPO_ROOT/$O/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --configs c2 --steps 1 > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1 || exit $?
echo pmc done
