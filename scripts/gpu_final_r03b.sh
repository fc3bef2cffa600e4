#!/bin/bash
# closing evidence (round 3, after the device integrals): full GPU suite + config tests, configs incl. c5dm32, smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_round.sh r03close nobench || exit 1
STEPS=configs,smoke CONFIGS=c5dm,c5dm32 bash scripts/gpu_final.sh || exit 1
