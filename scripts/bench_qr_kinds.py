"""Time the tall unpivoted QR factorizations the PT generator's right-canonical sweep needs (shapes taken from
scripts/bench_ptgen.py --stats, biexciton K = 205): pyaceqd_amd's Householder kernels (ptgen_gpu.qr_cols), a shifted
Cholesky-QR3 built from library GEMM / triangular solves, and torch.linalg.qr. Prints time, orthogonality and
residual for each. usage: python scripts/bench_qr_kinds.py"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from pyaceqd_amd import ptgen_gpu  # noqa: E402

SHAPES = [(2955, 636), (1365, 384), (915, 372), (640, 273), (450, 183), (200, 60), (96, 40), (60, 20)]
if os.environ.get("QK_SHAPES"):  # e.g. QK_SHAPES=2955x636,640x273
    SHAPES = [tuple(int(v) for v in s.split("x")) for s in os.environ["QK_SHAPES"].split(",")]


def cholqr3(W):
    m, n = W.shape
    u = 2.0 ** -53
    nrm2 = float(torch.linalg.vector_norm(W)) ** 2
    s = 11.0 * (m * n + n * (n + 1)) * u * nrm2
    G = W.conj().T @ W
    G.diagonal().add_(s)
    R1, _ = torch.linalg.cholesky_ex(G, upper=True)
    Q = torch.linalg.solve_triangular(R1, W, upper=True, left=False)
    R = R1
    for _ in range(2):
        G = Q.conj().T @ Q
        Rk, _ = torch.linalg.cholesky_ex(G, upper=True)
        Q = torch.linalg.solve_triangular(Rk, Q, upper=True, left=False)
        R = Rk @ R
    return Q, R


def ours(W):
    Qc, Rc, _, k = ptgen_gpu.qr_cols(W.T.contiguous())
    return Qc.T, Rc.T


def blocked(W):
    os.environ["PQD_PTG_BLOCKED"] = "1"
    try:
        return ours(W)
    finally:
        os.environ["PQD_PTG_BLOCKED"] = "0"


def wave(W):
    os.environ["PQD_PTG_WG"] = "0"
    os.environ["PQD_PTG_QFB"] = "0"
    try:
        return ours(W)
    finally:
        os.environ["PQD_PTG_WG"] = "1"
        os.environ["PQD_PTG_QFB"] = "1"


def lib(W):
    return torch.linalg.qr(W)


def small_shapes():
    """single-workgroup QR (m * n <= 8192, n <= 256) per shape, plain and pivoted"""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(2)
    for m, n in [(15, 45), (30, 90), (60, 120), (40, 200), (100, 40), (200, 40), (128, 64), (64, 128), (300, 27)]:
        W = torch.randn(n, m, dtype=torch.complex128, generator=g).to(dev)
        for piv in (False, True):
            for _ in range(3):
                ptgen_gpu.qr_cols(W, pivot=piv, tol=-1e-12)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                ptgen_gpu.qr_cols(W, pivot=piv, tol=-1e-12)
            torch.cuda.synchronize()
            print(f"small {m:4d} x {n:4d} pivot={int(piv)} {(time.perf_counter() - t0) / 50 * 1e6:8.1f} us", flush=True)


def main():
    if os.environ.get("QK_SMALL"):
        small_shapes()
        return
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    for m, n in SHAPES:
        # graded spectrum down to 1e-12 like a canonical-sweep matrix
        A = torch.randn(m, n, dtype=torch.complex128, generator=g)
        U, _ = torch.linalg.qr(A)
        V, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.complex128, generator=g))
        s = torch.logspace(0, -12, n, dtype=torch.float64)
        W = ((U * s) @ V.conj().T).to(dev)
        kinds = (("wave", wave), ("householder", ours), ("blocked", blocked), ("torch.qr", lib))
        if os.environ.get("QK_KINDS"):
            kinds = [k for k in kinds if k[0] in os.environ["QK_KINDS"].split(",")]
        for name, f in kinds:
            for _ in range(2):
                Q, R = f(W)
            torch.cuda.synchronize()
            reps = 5 if m * n > 50000 else 20
            t0 = time.perf_counter()
            for _ in range(reps):
                Q, R = f(W)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            orth = float(torch.linalg.matrix_norm(Q.conj().T @ Q - torch.eye(Q.shape[1], dtype=Q.dtype, device=dev)))
            res = float(torch.linalg.matrix_norm(Q @ R - W) / torch.linalg.matrix_norm(W))
            print(f"{m:5d} x {n:4d} {name:12s} {dt * 1e3:9.3f} ms  |Q^H Q - I| {orth:.1e}  |QR - W|/|W| {res:.1e}",
                  flush=True)


main()
