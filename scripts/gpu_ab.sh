#!/bin/bash
# A/B of sweep-kernel variants on the bench workload (no CPU baseline). Each variant is one bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  i=$((i+1))
  echo "== variant $i: $v"
  ve=${v%%|*}; va=""; [[ $v == *"|"* ]] && va=${v#*|}   # "ENV=.. ENV=.. | bench args"
  env $ve timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} $va > gpurun_out/ab_$i.log 2>&1
  rc=$?; echo "rc=$rc"; grep -o '"value": [0-9.e+]*\|"pt_sweep": [0-9.]*\|"frac": [0-9.]*' gpurun_out/ab_$i.log | tr '\n' ' '; echo
  if crash $rc; then tail -20 gpurun_out/ab_$i.log; exit $rc; fi
done <<< "${VARIANTS:-PQD_PT_MODE=4 PQD_CMUL3=1
PQD_PT_MODE=1 PQD_CMUL3=0
PQD_PT_MODE=4 PQD_CMUL3=0
PQD_PT_MODE=1 PQD_CMUL3=1}"
exit 0
