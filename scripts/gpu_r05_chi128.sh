#!/bin/bash
# round 5: the chi = 128 dictionary workload (the shape of the generated biexciton PT at the
# reference parameters): timings, rocprofv3 kernel stats, one SQ counter pass; then the generated-PT row itself
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/chi128
mkdir -p $O
export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$O/$name.log" | cut -c1-900; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; }
run cfg 400 python3 -u scripts/bench_configs.py --configs c4d128s,c4d128,c3d ${EXTRA:-}
run trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/bench_configs.py --configs c4d128s --steps 1
run pmc 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc -o run --output-format csv -- python3 scripts/bench_configs.py --configs c4d128s --steps 1
[ -n "$GEN" ] && run gen 600 python3 -u scripts/bench_configs.py --configs c4g --steps 2
exit 0
