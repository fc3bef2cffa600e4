"""Per-step cost of the host PT generator (pyaceqd_amd/ptgen.py) at the biexciton defaults of
general_system.py:152-211 (boson op diag(0,1,1,2), t_mem 20.48 ps, threshold 1e-10) at dt = 0.1 ps (K = 205).
usage: python scripts/prof_ptgen.py [--steps N] [--dt DT] [--profile] [--threads T]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--dt", type=float, default=0.1)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--threshold", type=float, default=1e-10)
    ap.add_argument("--tmem", type=float, default=20.48)
    ap.add_argument("--save", default=None, help="write the slices to this .npz (for comparisons)")
    a = ap.parse_args()
    import numpy as np
    from pyaceqd_amd import ptgen
    B = np.diag([0.0, 1.0, 1.0, 2.0]).astype(np.complex128)
    n_mem = max(1, int(round(a.tmem / a.dt)))
    J = lambda w: ptgen.qd_phonon_J(w, ae=3.0)  # noqa: E731
    eta, delta = ptgen.eta_coefficients(J, 1.0, a.dt, n_mem, e_max=7.0)
    b = ptgen.GaussianPTBuilder(B, eta, delta, a.dt, threshold=a.threshold, max_bond=64)
    pr = cProfile.Profile() if a.profile else None
    t_all = time.perf_counter()
    Qs = []
    for n in range(a.steps):
        t0 = time.perf_counter()
        if pr is not None and n >= a.steps - 5:
            pr.enable()
        Q, c = b.step()
        if pr is not None:
            pr.disable()
        Qs.append(Q)
        tails = [t.shape[2] for t in b.tail[:-1]]
        print(f"step {n + 1:4d} {time.perf_counter() - t0:7.3f} s  bond {b.r:3d}  tail max {max(tails or [1]):3d}",
              flush=True)
    print(f"total {time.perf_counter() - t_all:.2f} s for {a.steps} steps (K = {b.K})", flush=True)
    if a.save:
        chi = max(max(q.shape[1], q.shape[2]) for q in Qs)
        Qp = np.zeros((len(Qs), Qs[0].shape[0], chi, chi), dtype=np.complex128)
        for s, q in enumerate(Qs):
            Qp[s, :, :q.shape[1], :q.shape[2]] = q
        np.savez(a.save, Q=Qp)
    if pr is not None:
        pstats.Stats(pr).sort_stats("cumulative").print_stats(18)


main()
