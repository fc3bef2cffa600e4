#!/bin/bash
# round 5: kernel statistics of the generator (bx01, N steps), only the summary comes back (the trace is > 64 MiB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05/qprof${TAG:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/qprof -o run --output-format csv -- python3 -u scripts/bench_ptgen.py --case bx01 --steps ${STEPS:-60} > $O/prof.log 2>&1
rc=$?
grep RESULT $O/prof.log
f=$(find /tmp/qprof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("total kernel ms", tot / 1e6, "calls", sum(int(r['Calls']) for r in rows))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):8d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:80]}")
PY
rm -rf /tmp/qprof
exit $rc
