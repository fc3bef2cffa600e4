"""Phase timing of the register-resident TLS sweep (pt_quad.hip) from in-kernel s_memtime stamps.

A diagnostic instantiation of the kernel (PQD_ABLATE bit 32) records s_memtime in workgroup 0, wave 0 at the
phase boundaries of steps 1000..1015; this prints the mean shader cycles of each phase.
  0 top -> 1 closure partial -> 2 column phase A -> 3 exchange + barrier -> 4 traces -> 5 PT contraction (results
  consumed) -> 6 operand loads issued -> 7 D -> C relayout -> 8 column phase B; step = 0 -> next 0
usage: python scripts/quad_stamps.py [--config c2] [--n-tau 2000]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "scripts"))

NAMES = ["partial", "colA", "exch+barrier", "traces", "PT", "loads", "relayout", "colB"]
FAST = ["partial+colA", "exch+barrier", "A+PT issue+traces+loads", "PT results", "relayout", "reload check"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n-tau", type=int, default=2000)
    args = ap.parse_args()
    import bench_configs
    from pyaceqd_amd import _lib, engine
    cfg = dict(bench_configs.CONFIGS[args.config], n_tau=args.n_tau)
    N, sysd, grid, pt, rho0, ops, tr = bench_configs.workload(**cfg)
    os.environ["PQD_ABLATE"] = "32"
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    os.environ.pop("PQD_ABLATE")
    plan.execute()
    plan.synchronize()
    plan.execute(rebuild_free=False)
    plan.synchronize()
    buf = (C.c_ulonglong * 256)()
    fn = _lib.lib().pqd_debug_quad_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    st = np.array(buf[:256], dtype=np.int64).reshape(16, 16)
    fast = st[0, 7] == 0 and st[0, 8] == 0  # the fast step writes slots 0..6
    names = FAST if fast else NAMES
    st = st[:, :len(names) + 1]
    ph = np.diff(st, axis=1)
    step = np.diff(st[:, 0])
    print(f"{args.config}: mean shader cycles per step {step.mean():.0f} (min {step.min()}, max {step.max()})")
    print("fast step" if fast else "general step")
    for k, nm in enumerate(names):
        print(f"  {nm:14s} {ph[:, k].mean():8.0f}   min {ph[:, k].min():6d}  max {ph[:, k].max():6d}")
    print(f"  {'(end -> next 0)':14s} {(st[1:, 0] - st[:-1, -1]).mean():8.0f}")


if __name__ == "__main__":
    main()
