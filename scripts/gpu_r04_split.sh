#!/bin/bash
# round 4: split-group granule exchange: parity, then C3 single-run latency A/B (granules vs counter)
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu \
    -k "split or config3" > gpurun_out/r04/pytest_split.log 2>&1 || { tail -40 gpurun_out/r04/pytest_split.log; exit 1; }
tail -3 gpurun_out/r04/pytest_split.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_robustness.py -x -v --timeout 200 --timeout-method thread -m gpu \
    -k "config3 or split" > gpurun_out/r04/pytest_split2.log 2>&1 || { tail -40 gpurun_out/r04/pytest_split2.log; exit 1; }
tail -3 gpurun_out/r04/pytest_split2.log
for r in 1 2; do
  for g in 1 0; do
    PQD_SPLIT_GRAN=$g timeout -k 10 200 python -u scripts/bench_configs.py --configs c3one --steps 3 > gpurun_out/r04/c3one_gran$g.$r.log 2>&1 || { tail -20 gpurun_out/r04/c3one_gran$g.$r.log; exit 1; }
    echo "gran=$g run $r"; grep -i "c3one" gpurun_out/r04/c3one_gran$g.$r.log | tail -2
  done
done
