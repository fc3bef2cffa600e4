#!/bin/bash
# GPU-box run: pytest -m gpu, smoke, bench. Every GPU step has its own time limit; a crash-class exit
# (timeout/abort/segfault/kill) ends the script; plain test failures (rc=1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name (limit ${lim}s)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; return 0; }
STEPS=${STEPS:-pytest,smoke,bench}
[[ $STEPS == *pytest* ]] && run pytest_gpu 1200 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS}
exit 0
