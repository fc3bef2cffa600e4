#!/bin/bash
# round-4 closing evidence: config tests + whole -m gpu suite + bench, then the rocprof kernel trace of the bench
# command, the SURVEY configurations and smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_round.sh r04b || exit 1
STEPS=trace,configs,smoke CONFIGS=c1,c2,c2one,c3one,c5,c5d,c3d bash scripts/gpu_final.sh || exit 1
