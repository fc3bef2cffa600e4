#!/bin/bash
# GPU-box run: bench sweep time at several n_tau (per-step cost of the distinct-slice region vs the repeated region).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ntau
for nt in ${NTAUS:-400 800 1600}; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --n-tau $nt > gpurun_out/ntau/n$nt.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ntau/n$nt.log') if x.startswith('{')][-1])
c=d['config']
print('n_tau', $nt, 'grid_steps', c['grid_steps'], 'sweep ms', round(c['kernel_ms']['pt_sweep'],3), 'us/step', round(1e3*c['kernel_ms']['pt_sweep']/c['grid_steps'],3))"
done
