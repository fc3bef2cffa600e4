cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/qv1; mkdir -p $O; export TMPDIR=/tmp
PQD_LIB=abq/libpqd_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_quad.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for L in pyaceqd_amd/libpqd.so abq/libpqd_v1.so; do
    PQD_LIB=$L timeout -k 10 120 python scripts/bench_configs.py --configs c2 --steps 5 > $O/q.log 2>&1 || { tail $O/q.log; exit 1; }
    echo "round $r $L: $(grep -o '"pt_sweep_ms": [0-9.]*\|"frac_fp64": [0-9.]*' $O/q.log | tr '\n' ' ')"
  done
done
