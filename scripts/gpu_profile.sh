#!/bin/bash
# GPU-box profiling: ablations + rocprofv3 kernel-trace stats of the bench command (+ optional PMC pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; }
STEPS=${STEPS:-ablate,trace}
[[ $STEPS == *ablate* ]] && run ablate 600 python scripts/profile_sweep.py ${ABL_ARGS}
[[ $STEPS == *trace* ]] && run rocprof_trace 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}
[[ $STEPS == *pmc* ]] && run rocprof_pmc 900 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/prof/pmc -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS}
[[ $STEPS == *bench* ]] && run bench 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_FULL_ARGS}
find gpurun_out/prof -name "*.csv" | head -20
exit 0
