#!/bin/bash
# GPU-box run: scripts/bench_configs.py on the current library and (if ab/libpqd_prev.so exists) on a previous
# build (or, with PREV_ENV="VAR=value ...", under those settings), for A/B of kernel changes on the
# non-headline configs. CONFIGS selects the configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-c5,c3one,c2}
timeout -k 10 300 python -u scripts/bench_configs.py --configs "$CONFIGS" > gpurun_out/cfg_new.log 2>&1
rc=$?; echo "== new rc=$rc"; cat gpurun_out/cfg_new.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$PREV_ENV" ]; then
  env $PREV_ENV timeout -k 10 300 python -u scripts/bench_configs.py --configs "$CONFIGS" > gpurun_out/cfg_prev.log 2>&1
  rc=$?; echo "== $PREV_ENV rc=$rc"; cat gpurun_out/cfg_prev.log
elif [ -f ab/libpqd_prev.so ]; then
  PQD_LIB=ab/libpqd_prev.so timeout -k 10 300 python -u scripts/bench_configs.py --configs "$CONFIGS" > gpurun_out/cfg_prev.log 2>&1
  rc=$?; echo "== prev rc=$rc"; cat gpurun_out/cfg_prev.log
fi
exit $rc
