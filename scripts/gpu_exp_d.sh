#!/bin/bash
set -o pipefail
O=gpurun_out/exp_d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mapchain or sweep_pt_contraction or config_workloads" tests/test_gpu_configs.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python -u scripts/bench_mapchain.py --cases onetime,block > $O/mc.log 2>&1 || { echo mc failed; tail $O/mc.log; exit 1; }
grep case $O/mc.log
timeout -k 10 300 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 4,5,6 --variants 0 --rounds 3 > $O/c5_ptmode.log 2>&1 || { echo c5 failed; tail $O/c5_ptmode.log; exit 1; }
grep sweep $O/c5_ptmode.log
timeout -k 10 300 python -u scripts/profile_sweep.py --config c5d --n-tau 1000 --pt-modes 4,5,6 --variants 0 --rounds 3 > $O/c5d_ptmode.log 2>&1 || { echo c5d failed; tail $O/c5d_ptmode.log; exit 1; }
grep sweep $O/c5d_ptmode.log
