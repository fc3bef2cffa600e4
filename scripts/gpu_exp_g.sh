#!/bin/bash
set -o pipefail
O=gpurun_out/exp_g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=15 -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit 1;; esac
timeout -k 10 400 python -u scripts/bench_mapchain.py --cases onetime,block,ft8,tlmap > $O/mc.log 2>&1 || { echo mc failed; tail $O/mc.log; exit 1; }
grep case $O/mc.log | cut -c1-400
PQD_LIB=ab/libpqd_base.so timeout -k 10 200 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0 --rounds 2 > $O/c5b.log 2>&1; echo "c5 base: $(grep sweep $O/c5b.log)"
timeout -k 10 200 python -u scripts/profile_sweep.py --config c5 --n-tau 1000 --pt-modes 5 --variants 0 --rounds 2 > $O/c5.log 2>&1; echo "c5 tree: $(grep sweep $O/c5.log)"
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -c 300 $O/bench.log
