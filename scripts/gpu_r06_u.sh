#!/bin/bash
# round 6: the C4 config tests with multi-trajectory split groups forced (PQD_MSPLIT=2), off (0) and in auto mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-u}
mkdir -p $O
for m in 2 0 1; do
  PQD_MSPLIT=$m timeout -k 10 300 python3 -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -k "config4" > $O/pytest_c4_ms$m.log 2>&1
  rc=$?; echo "PQD_MSPLIT=$m rc=$rc: $(tail -1 $O/pytest_c4_ms$m.log)"
  case $rc in 0|1) ;; *) exit 1;; esac
done
exit 0
