#!/bin/bash
# round 4: split groups dealt onto one XCD per group (PQD_SPLIT_XCD): parity, then C3 single-run A/B x exchange form
set -o pipefail
mkdir -p gpurun_out/r04/xcd
export PYTHONUNBUFFERED=1
T=gpurun_out/r04/xcd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu \
    -k "split or config3" > $T/pytest_split_xcd.log 2>&1 || { tail -40 $T/pytest_split_xcd.log; exit 1; }
tail -2 $T/pytest_split_xcd.log
for r in 1 2; do
  for x in 1 0; do
    for g in 1 0; do
      PQD_SPLIT_XCD=$x PQD_SPLIT_GRAN=$g timeout -k 10 200 python -u scripts/bench_configs.py --configs c3one --steps 3 > $T/c3one_x${x}_g${g}.$r.log 2>&1 || { tail -20 $T/c3one_x${x}_g${g}.$r.log; exit 1; }
      echo "xcd=$x gran=$g run $r: $(grep -i "c3one" $T/c3one_x${x}_g${g}.$r.log | tail -1 | cut -c1-200)"
    done
  done
done
