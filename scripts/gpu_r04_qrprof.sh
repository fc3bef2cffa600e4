#!/bin/bash
# kernel statistics of the plain QR variants on the largest right-canonical block (2955 x 636)
set -o pipefail
mkdir -p gpurun_out/r04
T=gpurun_out/r04
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in householder blocked; do
  QK_SHAPES=2955x636 QK_KINDS=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_qr_$k -o qr -- python3 scripts/bench_qr_kinds.py > $T/qrprof_$k.log 2>&1 || { tail -20 $T/qrprof_$k.log; exit 1; }
  find /tmp/prof_qr_$k -name "*kernel_stats*" -exec cp {} $T/qrprof_${k}_kernel_stats.csv \;
  grep -E "ms " $T/qrprof_$k.log
  cut -c1-200 $T/qrprof_${k}_kernel_stats.csv | head -12
done
