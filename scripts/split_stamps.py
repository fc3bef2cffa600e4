"""Phase timing of the split-group latency path (pt_split.hip, the C3 single run) from in-kernel s_memtime stamps.

A diagnostic instantiation of the kernel (PQD_ABLATE bit 32; counter exchange, N2 = 16, chi = 64) records s_memtime
in workgroups 0 and G-1 of the group (thread 0) at the phase boundaries of steps 1000..1015 (G-1 is the output
workgroup, G = 17, unless PQD_SPLIT_OW=0 / --ow 0: then G = 16 and workgroup 0 writes the outputs); this prints the
mean shader cycles of each phase:
  0 top -> 1 column phase (row g of F(n) X) -> 2 PT row partials -> 3 row published (sc1 stores, drain, barrier,
  counter add) -> 4 output (workgroup 0) + next operator row fetch -> 5 peers arrived (poll + barrier) ->
  6 state gathered (16 KiB sc1 loads + barrier); step = 0 -> next 0
usage: python scripts/split_stamps.py [--n-tau 2000] [--ow 0|1]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "scripts"))

NAMES = ["column (F row)", "PT row", "publish+arrive", "output+fetch", "poll peers", "gather"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-tau", type=int, default=2000)
    ap.add_argument("--ow", type=int, default=1, help="0: no output workgroup (PQD_SPLIT_OW=0)")
    args = ap.parse_args()
    if args.ow == 0:
        os.environ["PQD_SPLIT_OW"] = "0"
    last = "workgroup 15" if args.ow == 0 else "workgroup 16 (output)"
    import bench_configs
    from pyaceqd_amd import _lib, engine
    cfg = dict(bench_configs.CONFIGS["c3one"], n_tau=args.n_tau)
    N, sysd, grid, pt, rho0, ops, tr = bench_configs.workload(**cfg)
    os.environ["PQD_ABLATE"] = "32"
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    os.environ.pop("PQD_ABLATE")
    plan.execute()
    plan.synchronize()
    plan.execute(rebuild_free=False)
    plan.synchronize()
    buf = (C.c_ulonglong * 256)()
    fn = _lib.lib().pqd_debug_split_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    st = np.array(buf[:256], dtype=np.int64).reshape(2, 16, 8)
    for w, name in enumerate(("workgroup 0", last)):
        s = st[w, :, :7].copy()
        # a phase the workgroup does not run (the output workgroup: no PT row, no publish) has no stamp: fold it into
        # the next phase
        for k in range(5, 0, -1):
            if np.all(s[:, k] == 0):
                s[:, k] = s[:, k - 1]
        ph = np.diff(s, axis=1)
        step = np.diff(s[:, 0])
        print(f"{name}: mean shader cycles per step {step.mean():.0f} (min {step.min()}, max {step.max()})")
        for k, nm in enumerate(NAMES):
            if np.all(st[w, :, k + 1] == 0):
                print(f"  {nm:16s}        -")
                continue
            print(f"  {nm:16s} {ph[:, k].mean():8.0f}   min {ph[:, k].min():6d}  max {ph[:, k].max():6d}")
        print(f"  {'(end -> next 0)':16s} {(s[1:, 0] - s[:-1, -1]).mean():8.0f}")
    for w, name in enumerate(("workgroup 0", last)):
        o = st[w]
        if np.all(o[:, 7] > 0):
            print(f"{name} output pass: operands staged + barrier {np.mean(o[:, 7] - o[:, 3]):.0f}, "
                  f"closure + traces + next fetch {np.mean(o[:, 4] - o[:, 7]):.0f}")


if __name__ == "__main__":
    main()
