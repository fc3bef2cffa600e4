#!/bin/bash
# single-workgroup QR: shape histogram in the generator and per-shape timings
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 200 python -u scripts/bench_ptgen.py --case bx01 --steps 25 --stats > $T/stats_bx01_small.log 2>&1 || { tail -20 $T/stats_bx01_small.log; exit 1; }
grep -E "SMALL|RESULT" $T/stats_bx01_small.log
QK_SMALL=1 timeout -k 10 120 python -u scripts/bench_qr_kinds.py > $T/qr_small_shapes.log 2>&1 || { tail -20 $T/qr_small_shapes.log; exit 1; }
cat $T/qr_small_shapes.log
