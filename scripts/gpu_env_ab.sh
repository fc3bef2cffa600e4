#!/bin/bash
# GPU-box run: scripts/bench_configs.py once per environment setting, alternating, for A/B of runtime switches.
# ENVS="A=1 B=2|A=0|" (settings separated by '|', an empty entry = defaults), CONFIGS, ROUNDS (default 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-c2}
ROUNDS=${ROUNDS:-2}
IFS='|' read -r -a SETS <<< "${ENVS:-}"
[ ${#SETS[@]} -eq 0 ] && SETS=("")
for r in $(seq 1 "$ROUNDS"); do
  for e in "${SETS[@]}"; do
    echo "== round $r env [$e]"
    env $e timeout -k 10 300 python -u scripts/bench_configs.py --configs "$CONFIGS" > gpurun_out/envab.tmp 2>&1
    rc=$?
    cat gpurun_out/envab.tmp
    [ $rc -ne 0 ] && { echo "rc=$rc: stopping"; exit $rc; }
  done
done
exit 0
