"""Fold a rocprofv3 --pmc pass of SQ_INSTS_VALU_MFMA_MOPS_F64 / SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES /
GRBM_GUI_ACTIVE (scripts/gpu_pmc.sh STEPS=mfma) into the executed-MFMA figures of one kernel.

  executed MFMA flop   = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (the counter's unit)
  effective clock      = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall (MI355X_MICROARCH.md, DVFS paragraph)
  MFMA-busy fraction   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)

usage: python scripts/pmc_mfma.py run_counter_collection.csv kernel_substring out.json [--peak 78.6]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("kernel")
    ap.add_argument("out")
    ap.add_argument("--peak", type=float, default=78.6)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    agg = collections.defaultdict(float)
    span = {}
    name = None
    for r in csv.DictReader(open(a.csv)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        span[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    wall_s = sum(span.values()) * 1e-9
    flop = agg["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
    cyc = agg["GRBM_GUI_ACTIVE"] / 8
    rec = {"kernel": name, "dispatches": len(span), "wall_ms": wall_s * 1e3,
           "counters": dict(agg),
           "executed_mfma_flop": flop,
           "executed_mfma_TFLOPs": flop / wall_s / 1e12,
           "executed_mfma_frac_of_peak": flop / wall_s / 1e12 / a.peak,
           "effective_clock_GHz": cyc / wall_s / 1e9,
           "mfma_busy_frac": agg["SQ_VALU_MFMA_BUSY_CYCLES"] / (a.simds * cyc) if cyc else None}
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
