#!/bin/bash
# round-6 evidence on the current head: config tests + whole -m gpu suite + bench, the rocprof kernel trace of the
# bench command, the MFMA counter pass of one full bench launch, smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_round.sh ${TAG:-r06/final} || exit 1
STEPS=trace,smoke bash scripts/gpu_final.sh || exit 1
STEPS=mfma PMC_BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline" bash scripts/gpu_pmc.sh || exit 1
exit 0
