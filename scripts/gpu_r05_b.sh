#!/bin/bash
# round 5: split-kernel phase stamps (C3 single run), then the round-5 evidence pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r05/split
timeout -k 10 200 python3 -u scripts/split_stamps.py --n-tau 2000 > gpurun_out/r05/split/stamps.log 2>&1
rc=$?; cat gpurun_out/r05/split/stamps.log | tail -22
case $rc in 0|1) ;; *) echo "stamps rc=$rc: stopping"; exit 1;; esac
TAG=r05b bash scripts/gpu_final_r05.sh
