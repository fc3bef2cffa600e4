"""Fold the separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes (scripts/gpu_pmc.sh STEPS=fetch,write, bench
config) into profiles/pmc_traffic.json, which bench.py reports as roofline.traffic for that config.

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE counts half the bytes of
16-B-per-lane streaming reads -> x2; WRITE_SIZE is exact for 16-B stores. Both counters are in KB.
usage: python scripts/pmc_traffic.py gpurun_out/pmc profiles/r01 [n_tau traj chi scan t1]"""
import csv
import json
import os
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    cfg = [int(x) for x in sys.argv[3:8]] if len(sys.argv) >= 8 else [10000, 2048, 64, 8, 256]
    out = {}
    for k, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        rows = [r for r in csv.DictReader(open(os.path.join(src, k, "run_counter_collection.csv")))
                if "pt_sweep" in r["Kernel_Name"]]
        out[c + "_KB"] = sum(float(r["Counter_Value"]) for r in rows)
        with open(os.path.join(dst, f"pmc_{k}_full.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    rec = {"kernel": "pt_sweep_kernel<16,64,8>",
           "config": dict(zip(["n_tau", "traj_per_gpu", "chi", "scan_points_per_gpu", "t1_points"], cfg)),
           "FETCH_SIZE_KB": out["FETCH_SIZE_KB"], "WRITE_SIZE_KB": out["WRITE_SIZE_KB"],
           "hbm_bytes_per_launch": out["FETCH_SIZE_KB"] * 1024 * 2 + out["WRITE_SIZE_KB"] * 1024,
           "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM/rocprofv3 section); WRITE_SIZE as reported; "
                         "units KB",
           "passes": "separate rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE runs of python bench.py "
                     "--steps 1 --warmup 0 --no-cpu-baseline",
           "source": "scripts/gpu_pmc.sh (STEPS=fetch,write) + scripts/pmc_traffic.py"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
