#!/bin/bash
# end-of-round evidence (round 3): config tests + GPU suite + bench line, kernel trace, other configs, smoke, PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_round.sh r03final || exit 1
STEPS=trace,configs,smoke CONFIGS=c1,c2,c2one,c3one,c5,c5d,c3d,c5dm,c4reuse bash scripts/gpu_final.sh || exit 1
PMC_BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline" STEPS=fetch,write,mfma bash scripts/gpu_pmc.sh || exit 1
