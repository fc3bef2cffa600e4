#!/bin/bash
# single-workgroup QR phases: kernel time with everything / without Q / without column steps
set -o pipefail
mkdir -p gpurun_out/r04/sd
T=gpurun_out/r04/sd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 0 1 3; do
  PQD_PTG_DIAG=$d QK_SMALL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sd$d -o sd -- python3 scripts/bench_qr_kinds.py > $T/sd$d.log 2>&1 || { tail -20 $T/sd$d.log; exit 1; }
  find /tmp/sd$d -name "*kernel_stats*" -exec cp {} $T/sd${d}_stats.csv \;
  find /tmp/sd$d -name "*kernel_trace*" -exec cp {} $T/sd${d}_trace.csv \;
done
ls -la $T
