#!/bin/bash
# C5 column tiles (4x4x4 vs 16x16 production builds vs the round-2-style single instance) and the headline kernel
set -o pipefail
O=gpurun_out/exp_f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "contraction_modes or config_workloads or sweep_pt or multi_system or mapchain" -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
for r in 1 2; do
  for lib in ab/libpqd_base.so ab/libpqd_col16.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$lib timeout -k 10 200 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0 --rounds 2 > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
    echo "c5 $lib: $(grep sweep $O/c5.log)"
  done
done
for r in 1 2; do
  for lib in ab/libpqd_base.so pyaceqd_amd/libpqd.so; do
    PQD_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
    echo "bench $lib: $(grep -o '"value": [0-9.e+]*\|"pt_sweep": [0-9.]*' $O/bench.log | tr '\n' ' ')"
  done
done
