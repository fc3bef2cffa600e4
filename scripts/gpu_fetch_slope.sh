#!/bin/bash
# GPU-box run: FETCH_SIZE of one bench sweep launch at several n_tau (traffic per step = slope), one pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/slope
export TMPDIR=/tmp
for nt in ${NTAUS:-2000 6000}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/slope/f$nt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --n-tau $nt ${EXTRA} > gpurun_out/slope/f$nt.log 2>&1 || exit $?
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('gpurun_out/slope/f$nt/run_counter_collection.csv')) if 'pt_sweep' in x['Kernel_Name']]
print('n_tau $nt FETCH_SIZE x2 GB', 2*sum(float(x['Counter_Value']) for x in r)/1e6)"
done
