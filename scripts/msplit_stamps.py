"""Phase timing of the multi-trajectory split groups (pt_msplit.hip) from in-kernel s_memtime stamps.

A diagnostic instantiation (PQD_ABLATE bit 64; N2 = 16, chi = 64) records s_memtime in workgroups 0 and 1 of group 0
(thread 0) at the phase boundaries of steps 1000..1015; this prints the mean shader cycles of each phase:
  0 top -> 1 PT partials + barrier -> 2 published (stores, drain, barrier, arrival word) -> 3 operands staged to
  LDS -> 4 peers arrived (poll + barrier) -> 5 gather loads + operand loads issued -> 6 the first chunk's loads back
  -> 7 gather done -> 8 end barrier; and per wave when the first chunk's loads are back and the gather is done
usage: python scripts/msplit_stamps.py [--n-t1 32] [--n-tau 2000]   (the C4 sweep shape, bench.build_workload)
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

NAMES = ["PT + barrier", "publish+arrive", "stage operands", "poll peers", "gather issue", "gather loads back",
         "gather compute", "end barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-t1", type=int, default=32)
    ap.add_argument("--n-tau", type=int, default=2000)
    ap.add_argument("--ablate", type=int, default=0, help="extra PQD_ABLATE bits (timing only: 128 no operand loads, 1024 gather loads at element 0, 2048 per-workgroup rotation of the gather order, 8192 gather loads of hardware half 1 at element 0)")
    args = ap.parse_args()
    import bench
    from pyaceqd_amd import _lib, engine
    sysd, grid, pt, rho0, ops, tr = bench.build_workload(args.n_t1, args.n_tau, 64, t1_offset=96)
    os.environ["PQD_ABLATE"] = str(64 | args.ablate)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    os.environ.pop("PQD_ABLATE")
    print("path", plan.info(), "ablate", args.ablate)
    plan.execute()
    plan.synchronize()
    plan.timing(reset=True)
    plan.execute(rebuild_free=False)
    plan.synchronize()
    _, ms, _ = plan.timing(reset=True)
    print(f"sweep {ms:.2f} ms, {ms * 1e3 / (grid.n_steps + 1):.3f} us per step")
    buf = (C.c_ulonglong * 1024)()
    fn = _lib.lib().pqd_debug_msplit_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    st = np.array(buf[:1024], dtype=np.int64).reshape(2, 16, 32)
    for w in range(2):
        s = st[w, :, :9]
        ph = np.diff(s, axis=1)
        step = np.diff(s[:, 0])
        print(f"workgroup {w}: mean shader cycles per step {step.mean():.0f} (min {step.min()}, max {step.max()})")
        for k, nm in enumerate(NAMES):
            print(f"  {nm:16s} {ph[:, k].mean():8.0f}   min {ph[:, k].min():6d}  max {ph[:, k].max():6d}")
        print(f"  {'(end -> next 0)':16s} {(s[1:, 0] - s[:-1, -1]).mean():8.0f}")
        for nm, b in (("loads back", 16), ("gather done", 24)):
            d = st[w, :, b:b + 8] - st[w, :, 4:5]  # cycles after the poll, waves 0..7
            print(f"  {nm} after the poll, waves 0..7:", " ".join(f"{v:.0f}" for v in d.mean(axis=0)))

if __name__ == "__main__":
    main()
