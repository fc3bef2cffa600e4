#!/bin/bash
# GPU-box run: SQ counters of the C2 quad-kernel sweep (scripts/bench_configs.py c2, one launch) for the default
# (8-column strips, one quad per workgroup) and the round-2-start setting (PQD_QPW=2 PQD_QCG=4). One --pmc pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc_c2
export TMPDIR=/tmp
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
for v in default old; do
  if [ $v = old ]; then export PQD_QPW=2 PQD_QCG=4; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/pmc_c2/$v -o run --output-format csv -- python3 scripts/bench_configs.py --configs c2 --steps 1 > gpurun_out/pmc_c2/$v.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections
for v in ("default", "old"):
    rows = [r for r in csv.DictReader(open(f"gpurun_out/pmc_c2/{v}/run_counter_collection.csv")) if "pt_quad" in r["Kernel_Name"]]
    tot = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    k = max(n.values()) if n else 1
    avg = {c: tot[c] / n[c] for c in tot}
    wc = avg.get("SQ_WAVE_CYCLES", 1)
    print(v, "launches", k, {c: round(avg[c] / 1e6, 3) for c in sorted(avg)})
    print(v, "wait share %.3f  inst-stall share %.3f  active share %.3f" % (avg.get("SQ_WAIT_ANY", 0) / wc,
          avg.get("SQ_WAIT_INST_ANY", 0) / wc, avg.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
