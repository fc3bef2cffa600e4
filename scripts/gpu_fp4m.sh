#!/bin/bash
# N2 = 4 free propagators on the matrix cores (libpqd.so) vs the shuffle products (ab/libpqd_base.so): parity, then
# C1 / C2 A/B in alternating rounds, then a kernel trace of the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/fp4m2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_robustness.py tests/test_gpu_quad.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; case $rc in 0) ;; *) grep -E "^FAILED|Error|assert" $O/pytest.log | head; echo "rc=$rc stop"; exit 1;; esac
for r in 1 2 3; do
  for L in ab/libpqd_base.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$L timeout -k 10 200 python scripts/bench_configs.py --configs c1,c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"config": "[a-z0-9]*"\|"wall_ms_per_launch": [0-9.]*\|"free_prop_ms": [0-9.]*' $O/q.log | tr '\n' ' ')" | tee -a $O/ab.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o c12 --output-format csv -- python3 scripts/bench_configs.py --configs c2,c1 --steps 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
# SQ counters of the C2 quad sweep (default setting), one --pmc pass
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d $O/pmc -o run --output-format csv -- python3 scripts/bench_configs.py --configs c2 --steps 1 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
