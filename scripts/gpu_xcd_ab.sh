#!/bin/bash
# GPU-box run: parity of the block-order change, then FETCH_SIZE / WRITE_SIZE of one bench launch and the bench line
# with the XCD-aware block order (default) and without (PQD_XCD=0). Each GPU step has its own time limit; a
# crash-class exit ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/xcd
export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/xcd/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "gpurun_out/xcd/$name.log"; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; }
run pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_branching.py tests/test_gpu_quad.py tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread
ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
for v in 1 0; do
  export PQD_XCD=$v
  run fetch_xcd$v 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/xcd/fetch$v -o run --output-format csv -- python3 bench.py $ARGS
  run write_xcd$v 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/xcd/write$v -o run --output-format csv -- python3 bench.py $ARGS
done
for r in 1 2; do for v in 1 0; do export PQD_XCD=$v; run bench_xcd${v}_$r 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline; done; done
exit 0
