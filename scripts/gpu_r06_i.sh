#!/bin/bash
# round 6: L2 hit rate and fabric traffic of the multi-trajectory split sweep (C4 shape, 256 t1), L2-kept vs sc1 stores
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r06/${TAG:-i}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for l2 in 1 0; do
  PQD_MS_L2=$l2 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O/pmc_hit_l2$l2 -- python3 $R/scripts/ms_prof.py > $R/$O/pmc_hit_l2$l2.log 2>&1 || exit 1
  PQD_MS_L2=$l2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch_l2$l2 -- python3 $R/scripts/ms_prof.py > $R/$O/pmc_fetch_l2$l2.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, os
O = os.environ.get("O_DIR", "gpurun_out/r06/i")
for f in sorted(glob.glob(O + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "msplit" in r.get("Kernel_Name", "")]
    agg = {}
    for r in rows:
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(f, {k: (len(v), sum(v) / len(v)) for k, v in agg.items()})
PY
exit 0
