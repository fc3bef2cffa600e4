#!/bin/bash
# A/B of whole source trees on the bench workload: ab/<name>/ holds an older tree's pyaceqd_amd/ (with its built
# libpqd.so) and bench.py; "cur" is this tree. Rounds alternate the variants so box drift hits all alike.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${TREES:-cur}; do
    name=${v%%:*}; envs=""; [[ $v == *:* ]] && envs=${v#*:}
    d=.; [ "$name" != cur ] && d=ab/$name
    (cd $d && env $envs timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS}) > gpurun_out/abt_${r}_${name}.log 2>&1
    rc=$?; printf "round %s %-24s rc=%s " "$r" "$v" "$rc"
    grep -o '"value": [0-9.e+]*\|"pt_sweep": [0-9.]*\|"frac": [0-9.]*\|"executed_traj_steps_per_gpu": [0-9]*' gpurun_out/abt_${r}_${name}.log | tr '\n' ' '; echo
    if crash $rc; then tail -20 gpurun_out/abt_${r}_${name}.log; exit $rc; fi
  done
done
exit 0
