#!/bin/bash
# the generator at the reference's defaults, GPU and the host restatement (NumPy/OpenBLAS on the box's 16 threads)
set -o pipefail
mkdir -p gpurun_out/r04
T=gpurun_out/r04
timeout -k 10 900 python -u scripts/bench_ptgen.py --case bx05,tls,sx05 --host > $T/bench_ptgen_host.log 2>&1 || { tail -20 $T/bench_ptgen_host.log; exit 1; }
grep RESULT $T/bench_ptgen_host.log
