#!/bin/bash
# round-3 re-entry evidence on the current head: config tests + whole -m gpu suite + bench, then the rocprof
# kernel trace of the bench command, the C2/C5 configurations and smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_round.sh r03f || exit 1
STEPS=trace,configs,smoke CONFIGS=c1,c2,c2one,c5,c3d bash scripts/gpu_final.sh || exit 1
