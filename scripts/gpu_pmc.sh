#!/bin/bash
# PMC passes for the sweep kernel (separate passes: FETCH_SIZE / WRITE_SIZE / SQ counters), plus the
# FP64 VALU-vs-MFMA overlap microbenchmark. No sys/runtime trace domains are combined with --pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 12 "gpurun_out/$name.log"; if crash $rc; then echo "crash-class exit: stopping"; exit $rc; fi; }
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --n-tau 2000}
STEPS=${STEPS:-ubench,fetch,write,sq}
if [[ $STEPS == *ubench* ]]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_fp64 scripts/ubench_fp64_pipes.hip && run ubench 120 /tmp/ubench_fp64
fi
[[ $STEPS == *fetch* ]] && run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run --output-format csv -- python bench.py $ARGS
[[ $STEPS == *write* ]] && run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run --output-format csv -- python bench.py $ARGS
[[ $STEPS == *sq* ]] && run pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc/sq -o run --output-format csv -- python bench.py $ARGS
[[ $STEPS == *list* ]] && run pmc_list 120 rocprofv3 -L
# executed-MFMA evidence for the headline kernel: FP64 MFMA ops, MFMA-busy cycles, SQ busy, clock
[[ $STEPS == *mfma* ]] && run pmc_mfma 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/mfma -o run --output-format csv -- python bench.py $ARGS
find gpurun_out/pmc -name "*counter_collection*.csv" | head
exit 0
