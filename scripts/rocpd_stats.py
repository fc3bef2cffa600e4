"""Kernel statistics from a rocprofv3 rocpd database (the default output format of ROCm 7.2's rocprofv3):
per kernel name calls / total / average duration (the columns of rocprofv3's kernel_stats.csv), plus, with --dispatches,
every dispatch of the kernels matching a pattern in launch order (grid, workgroup, duration).
usage: python scripts/rocpd_stats.py <results.db> [--out kernel_stats.csv] [--dispatches pt_msplit] [--dout file.csv]
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out")
    ap.add_argument("--dispatches")
    ap.add_argument("--dout")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]
    out = [[r[0], r[1], r[2], r[3], 100.0 * r[2] / tot, r[4], r[5]] for r in rows]
    if a.out:
        with open(a.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(out)
    for r in out[:12]:
        print(f"{r[3] / 1e6:10.3f} ms avg  {r[1]:5d} calls  {r[4]:5.1f}%  {r[0][:90]}")
    if a.dispatches:
        d = c.execute("select name, start, duration, grid_x, workgroup_x, lds_size, vgpr_count, accum_vgpr_count, "
                      "scratch_size from kernels where name like ? order by start", (f"%{a.dispatches}%",)).fetchall()
        for r in d:
            print(f"  {r[2] / 1e6:10.3f} ms  grid {r[3]} wg {r[4]} lds {r[5]} vgpr {r[6]}+{r[7]} scratch {r[8]}  {r[0][:60]}")
        if a.dout:
            with open(a.dout, "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["Name", "StartNs", "DurationNs", "GridX", "WorkgroupX", "LdsBytes", "VGPR", "AGPR", "Scratch"])
                w.writerows(d)


if __name__ == "__main__":
    main()
