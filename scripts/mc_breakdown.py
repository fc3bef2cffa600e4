"""Where the wall time of one calc_onetime_parallel call goes (C4 shape: 256 t1 x 10,000 tau steps): Python-side wall
per call next to libpqd's own phase times (PQD_MC_TIMING=1 prints upload+launch / page touch / kernels left /
download on stderr). usage: python scripts/mc_breakdown.py [--dim 4] [--reps 4]"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=4)
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    os.environ["PQD_MC_TIMING"] = "1"
    import bench_mapchain as B
    from pyaceqd_amd.two_time import propagate_tau_module as gpu
    dim, n_t, n_tau, dt = args.dim, 256, 10000, 0.1
    n_tfull = n_t + n_tau + 2
    dm = B._maps(n_tfull, dim, seed=dim)
    time_full = dt * np.arange(n_tfull)
    ts = time_full[:n_t] + 1e-9
    rho0 = np.zeros(dim * dim, complex)
    rho0[0] = 1
    A, Bo, C = B._ops(dim, 7)
    for _ in range(args.reps):
        t0 = time.perf_counter()
        out = gpu.calc_onetime_parallel(dm, rho0, n_tau, dim, A, Bo, C, time_full, ts)
        t1 = time.perf_counter()
        print(f"call {1e3 * (t1 - t0):.3f} ms", flush=True)
        del out
    t0 = time.perf_counter()
    z = np.zeros((n_t, n_tau + 1), dtype=np.complex128, order="F")
    z[::8] = 0
    print(f"np.zeros + touch of the result shape: {1e3 * (time.perf_counter() - t0):.3f} ms")


if __name__ == "__main__":
    main()
