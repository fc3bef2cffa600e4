#!/bin/bash
# Paterson-Stockmeyer free propagators: parity (free-propagator tests, configs), then C5 / headline timings
set -o pipefail
mkdir -p gpurun_out/r04/ps
T=gpurun_out/r04/ps
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "free" > $T/pytest_ps.log 2>&1 || { tail -40 $T/pytest_ps.log; exit 1; }
tail -2 $T/pytest_ps.log
timeout -k 10 600 python -u scripts/bench_configs.py --configs c5,c5d,c3d > $T/configs_ps.log 2>&1 || { tail -20 $T/configs_ps.log; exit 1; }
grep -E '"config"' $T/configs_ps.log | cut -c1-330
