#!/bin/bash
# round 5: headline kernel with its per-step metadata in registers (events, schedule, PT units) vs the previous build
# (pyaceqd_amd/libpqd_base.so through PQD_LIB), alternating runs on one box; parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/${TAG:-swmeta}
mkdir -p $O
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_configs.py -m gpu -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or branch or trunk or config3 or config4_g2_sweep_256_t1_full" > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0) ;; *) echo "parity rc=$rc: stopping"; exit 1;; esac
for r in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=pyaceqd_amd/libpqd_base.so; else L=; fi
    PQD_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$v.$r.log 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.$r.log) $(grep -o '"pt_sweep_ms[a-z_]*": [0-9.]*' $O/bench_$v.$r.log | head -1)"
  done
done
exit 0
