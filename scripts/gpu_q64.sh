#!/bin/bash
# chi = 64 TLS: quad (spilling first cut) vs batched; quad stamps at C2; map-chain after the page-touch overlap
set -o pipefail
O=gpurun_out/q64
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit 1;; esac
PQD_QUAD=0 timeout -k 10 200 python -u scripts/profile_sweep.py --config c2x64 --n-tau 2000 --variants 0 --rounds 2 > $O/b64.log 2>&1 || { tail $O/b64.log; exit 1; }
echo "batched chi64: $(grep sweep $O/b64.log)"
timeout -k 10 200 python -u scripts/profile_sweep.py --config c2x64 --n-tau 2000 --variants 0 --rounds 2 > $O/q64.log 2>&1 || { tail $O/q64.log; exit 1; }
echo "quad2 chi64: $(grep sweep $O/q64.log)"
timeout -k 10 100 python -u scripts/quad_stamps.py --config c2 > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 400 python -u scripts/bench_mapchain.py --cases onetime,block,ft8 > $O/mc.log 2>&1 || { echo mc failed; tail $O/mc.log; exit 1; }
grep case $O/mc.log | cut -c1-330
