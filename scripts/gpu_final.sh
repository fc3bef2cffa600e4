#!/bin/bash
# GPU-box end-of-round evidence: the default bench line (with its CPU baseline), a rocprofv3 kernel trace of the bench
# command, the other SURVEY configurations, smoke(). Every GPU step has its own time limit; a crash-class exit ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; }
STEPS=${STEPS:-bench,trace,configs,smoke}
[[ $STEPS == *bench* ]] && run bench 600 python3 bench.py
[[ $STEPS == *trace* ]] && run trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
[[ $STEPS == *configs* ]] && run configs 900 python3 -u scripts/bench_configs.py --configs ${CONFIGS:-c1,c2,c2one,c3one,c5,c5d,c3d,c5dm,c4reuse}
[[ $STEPS == *smoke* ]] && run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
exit 0
