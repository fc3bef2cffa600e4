"""Wall time of the PT generator (ACE's `dont_propagate` + `write_PT`, reference general_system.py:152-211) on the
GPU (pyaceqd_amd/ptgen_gpu.py) and, optionally, on the host (pyaceqd_amd/ptgen.py) for the same parameters.

cases (QD phonons, ae 3 nm unless stated, T 4 K, bond cap 128 for N <= 4):
  bx05   biexciton at the reference's defaults (four_level_system/linear.py:8): dt 0.5, t_mem 20.48 -> K = 41, 1e-10
  tls    TLS at the reference's defaults (tls.py:16): dt 0.1, t_mem 6.4 -> K = 64, ae 5 nm, threshold 1e-8
  bx01   biexciton at dt 0.1 (the bench's step): K = 205, 1e-10
  sx05   six-level at the reference's defaults (six_level_system/linear.py:28, 50, 67): dt 0.5, K = 41, 1e-10, bond cap 64
usage: python scripts/bench_ptgen.py [--case bx05,tls,bx01] [--steps N] [--host] [--tail qrcp|svd]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

CASES = {
    "bx05": dict(lam=[0, 1, 1, 2], dt=0.5, t_mem=20.48, ae=3.0, thr=1e-10),
    "tls": dict(lam=[0, 1], dt=0.1, t_mem=6.4, ae=5.0, thr=1e-8),
    "bx01": dict(lam=[0, 1, 1, 2], dt=0.1, t_mem=20.48, ae=3.0, thr=1e-10),
    "sx05": dict(lam=[0, 1, 1, 1, 1, 2], dt=0.5, t_mem=20.48, ae=3.0, thr=1e-10, cap=64),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="bx05,tls")
    ap.add_argument("--steps", type=int, default=0, help="stop after N steps (0: the whole PT, 2K + stationary)")
    ap.add_argument("--host", action="store_true", help="also time the host generator")
    ap.add_argument("--tail", default="qrcp")
    ap.add_argument("--stats", action="store_true", help="factorization shapes / Jacobi sweeps of the last step")
    a = ap.parse_args()
    if a.stats:
        os.environ["PQD_PTG_DEBUG"] = "1"
    import numpy as np
    from pyaceqd_amd import ptgen, ptgen_gpu
    for name in a.case.split(","):
        c = CASES[name]
        A = np.diag(np.array(c["lam"], dtype=float))
        K = int(round(c["t_mem"] / c["dt"]))
        J = lambda w: ptgen.qd_phonon_J(w, ae=c["ae"])  # noqa: E731
        eta, delta = ptgen.eta_coefficients(J, 4.0, c["dt"], K)
        for side in (["gpu", "host"] if a.host else ["gpu"]):
            if side == "gpu":
                b = ptgen_gpu.GaussianPTBuilderGPU(A, eta, delta, c["dt"], c["thr"], c.get("cap", 128), tail=a.tail)
                import torch
                sync = torch.cuda.synchronize
            else:
                b = ptgen.GaussianPTBuilder(A, eta, delta, c["dt"], c["thr"], c.get("cap", 128))
                sync = lambda: None  # noqa: E731
            n_tot = 2 * K if not a.steps else min(a.steps, 2 * K)
            t0 = time.perf_counter()
            tl = t0
            for n in range(n_tot):
                if a.stats and side == "gpu":
                    ptgen_gpu._STATS.clear()
                b.step()
                if n % 20 == 0 or n == n_tot - 1:
                    sync()
                    t = time.perf_counter()
                    tails = [int(x.shape[2]) for x in b.tail[:-1]]
                    print(f"{name} {side} step {n + 1}/{2 * K} {t - t0:8.2f} s (last block {t - tl:6.2f} s) "
                          f"bond {b.r} tail max {max(tails or [1])}", flush=True)
                    tl = t
            if a.stats and side == "gpu":
                import collections
                st = ptgen_gpu._STATS
                cnt = collections.Counter(x[0] for x in st)
                big = sorted((x for x in st if x[0] != "jacobi"), key=lambda x: -x[1] * x[2])[:12]
                print(f"STATS last step: {dict(cnt)}; jacobi (n, sweeps): {[x[1:] for x in st if x[0] == 'jacobi']}; "
                      f"largest QRs (m, n, rank): {[x[1:] for x in big]}; "
                      f"column steps: {sum(min(x[1], x[2]) if x[0] == 'qr' else x[3] for x in st if x[0] != 'jacobi')}",
                      flush=True)
                small = [x for x in st if x[0] != "jacobi" and x[1] * x[2] <= 8192 and x[2] <= 256]
                hist = collections.Counter((x[0], "wide" if x[1] < x[2] else "tall", min(x[1], 256) // 32 * 32,
                                            min(x[2], 256) // 32 * 32) for x in small)
                print(f"SMALL (single-workgroup) calls: {len(small)}; by (kind, shape, m//32*32, n//32*32): "
                      f"{sorted(hist.items(), key=lambda t: -t[1])[:24]}", flush=True)
            if n_tot == 2 * K:
                b.stationary_slice()
            sync()
            el = time.perf_counter() - t0
            full = el if n_tot == 2 * K else el * (2 * K + 1) / n_tot
            if side == "gpu":
                print(f"Jacobi retries (n, attempt): {ptgen_gpu.RETRIES}", flush=True)
                if ptgen_gpu._PHASES is not None:
                    print(f"PHASES (s, synchronised): {ptgen_gpu._PHASES}", flush=True)
            print(f"RESULT {name} {side} tail={a.tail} K={K} steps={n_tot} {el:.2f} s "
                  f"(whole PT {'measured' if n_tot == 2 * K else 'extrapolated'}: {full:.1f} s)", flush=True)


main()
