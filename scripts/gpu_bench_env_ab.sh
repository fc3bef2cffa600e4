#!/bin/bash
# GPU-box run: bench.py lines alternating between the defaults and ENV_B (e.g. "PQD_WIN=0"), ROUNDS rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/benchab
for r in $(seq 1 "${ROUNDS:-2}"); do
  for e in "" "$ENV_B"; do
    env $e timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/benchab/run.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/benchab/run.log') if x.startswith('{')][-1])
print('[$e]', round(d['value']/1e6,2), 'M/s sweep', round(d['config']['kernel_ms']['pt_sweep'],2), 'ms free', round(d['config']['kernel_ms']['free_prop'],2))"
  done
done
