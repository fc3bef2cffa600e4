#!/bin/bash
# 16-lane closure partials: parity (sweep / bench-workload / config tests), then bench A/B vs PQD_CLOS16=0 (3 rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r04/clos16
T=gpurun_out/r04/clos16
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "sweep or bench_workload or config3 or config4 or config5 or outputs or mto or trunk" > $T/pytest_clos16.log 2>&1 || { tail -40 $T/pytest_clos16.log; exit 1; }
tail -2 $T/pytest_clos16.log
ROUNDS=3 ENV_B="PQD_CLOS16=0" bash scripts/gpu_bench_env_ab.sh 2>&1 | tee $T/ab_clos16.log
