"""Fold three rocprofv3 SQ counter passes (scripts/gpu_r04_pmc_sq.sh / gpu_r05_pmc128.sh: sqA, sqB, sqC) of one kernel
into the cycle breakdown of DESIGN.md §7: MFMA-busy, non-MFMA VALU issue (4 cycles per wave64 instruction), the
remainder in which no wave of a SIMD issues, per-wave wait fractions and the LDS bank-conflict share.

usage: python scripts/pmc_breakdown.py <dir with sqA/ sqB/ sqC/> <kernel substring> out.json [--simds 1024]"""
import argparse
import collections
import csv
import glob
import json
import os


def fold(path, kernel):
    agg = collections.defaultdict(float)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("out")
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    A, B, C = (fold(os.path.join(a.dir, p), a.kernel) for p in ("sqA", "sqB", "sqC"))
    cyc = A["GRBM_GUI_ACTIVE"] / 8                      # kernel cycles per XCD (= per SIMD)
    valu_nonmfma = C["SQ_INSTS_VALU"] - C["SQ_INSTS_MFMA"]
    rec = {
        "kernel_cycles_per_xcd": cyc,
        "mfma_busy_frac": A["SQ_VALU_MFMA_BUSY_CYCLES"] / (a.simds * cyc),
        "valu_nonmfma_instr": valu_nonmfma,
        "valu_nonmfma_issue_frac (4 cycles each)": 4 * valu_nonmfma / (a.simds * cyc),
        "fp64_add_instr": C["SQ_INSTS_VALU_ADD_F64"],
        "fp64_fma_instr": C["SQ_INSTS_VALU_FMA_F64"],
        "mfma_valu_coexec_cycles": B["SQ_VALU_MFMA_COEXEC_CYCLES"],
        "lds_bank_conflict_over_lds_active": B["SQ_LDS_BANK_CONFLICT"] / max(B["SQ_LDS_IDX_ACTIVE"], 1),
        "per_wave_wait_any": A["SQ_WAIT_ANY"] / A["SQ_WAVE_CYCLES"],
        "per_wave_wait_inst_any": A["SQ_WAIT_INST_ANY"] / A["SQ_WAVE_CYCLES"],
        "per_wave_wait_inst_lds": B["SQ_WAIT_INST_LDS"] / B["SQ_WAVE_CYCLES"],
        "mfma_instr": C["SQ_INSTS_MFMA"],
        "lds_instr": C["SQ_INSTS_LDS"],
        "salu_instr": C["SQ_INSTS_SALU"],
    }
    rec["remainder_frac"] = 1 - rec["mfma_busy_frac"] - rec["valu_nonmfma_issue_frac (4 cycles each)"]
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
