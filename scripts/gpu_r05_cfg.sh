#!/bin/bash
# round 5: the other BASELINE configurations on the current head (bench_configs default set), two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/cfg
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 500 python3 -u scripts/bench_configs.py --configs ${CONFIGS:-c1,c2,c2one,c3one,c3eight,c5,c5one,c5d,c3d,c5dm,c4reuse} --steps 3 > $O/cfg_${TAG:-a}.$r.log 2>&1 || { tail -20 $O/cfg_${TAG:-a}.$r.log; exit 1; }
  grep -o '"config": "[a-z0-9]*"\|"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*\|"wall_ms_per_launch": [0-9.]*\|"free_prop_ms": [0-9.]*' $O/cfg_${TAG:-a}.$r.log | paste -s -d' ' | sed 's/"config"/\n"config"/g'
done
exit 0
