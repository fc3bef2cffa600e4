#!/bin/bash
# round 4 combined: generator tests + profile + timings, map tail, split granules (parity + C3 A/B)
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T=gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_ptgen.py -x -v --timeout 300 --timeout-method thread -m gpu > $T/pytest_ptgen.log 2>&1 || { tail -50 $T/pytest_ptgen.log; exit 1; }
tail -2 $T/pytest_ptgen.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_correlations_golden.py -x -v --timeout 200 --timeout-method thread -m gpu -k "map_tail or phonon_map" > $T/pytest_maptail.log 2>&1 || { tail -50 $T/pytest_maptail.log; exit 1; }
tail -2 $T/pytest_maptail.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robustness.py -x -v --timeout 200 --timeout-method thread -m gpu -k "split or config3" > $T/pytest_split.log 2>&1 || { tail -50 $T/pytest_split.log; exit 1; }
tail -2 $T/pytest_split.log
for r in 1 2; do for g in 1 0; do
  PQD_SPLIT_GRAN=$g timeout -k 10 200 python -u scripts/bench_configs.py --configs c3one --steps 3 > $T/c3one_gran$g.$r.log 2>&1 || { tail -20 $T/c3one_gran$g.$r.log; exit 1; }
  echo "gran=$g run $r: $(grep -i c3one $T/c3one_gran$g.$r.log | tail -1)"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ptgen -o ptg -- python3 scripts/bench_ptgen.py --case bx05 --steps 20 > $T/bench_ptgen_prof.log 2>&1 || { tail -30 $T/bench_ptgen_prof.log; exit 1; }
find /tmp/prof_ptgen -name "*stats*" -exec cp {} $T/ \;
ls $T | grep -i stat
timeout -k 10 300 python3 -m cProfile -s tottime scripts/bench_ptgen.py --case bx05 --steps 20 > $T/cprof_ptgen.log 2>&1 || { tail -30 $T/cprof_ptgen.log; exit 1; }
timeout -k 10 300 python3 -m cProfile -s tottime scripts/bench_ptgen.py --case bx01 --steps 30 > $T/cprof_ptgen_bx01.log 2>&1 || { tail -30 $T/cprof_ptgen_bx01.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_ptgen.py --case bx05,tls > $T/bench_ptgen.log 2>&1 || { tail -30 $T/bench_ptgen.log; exit 1; }
grep RESULT $T/bench_ptgen.log
timeout -k 10 400 python -u scripts/bench_ptgen.py --case bx01 --steps 80 > $T/bench_ptgen_bx01.log 2>&1 || { tail -30 $T/bench_ptgen_bx01.log; exit 1; }
grep RESULT $T/bench_ptgen_bx01.log
