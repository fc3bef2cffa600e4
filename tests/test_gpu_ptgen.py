"""GPU PT generator (pyaceqd_amd/ptgen_gpu.py + csrc/ptgen.hip; replaces ACE's `dont_propagate` + `write_PT`,
reference general_system.py:152-211).

  * the device factorizations against numpy/LAPACK: Householder QR (same reflector convention as zgeqrf, so R
    equals numpy's R), the rank-revealing column-pivoted QR, and the QR-preconditioned one-sided Jacobi SVD, on
    both the single-workgroup (LDS) and the multi-workgroup kernels;
  * the generated PT against the host generator ptgen.py in influence values (path contractions
    bond0 Q_1[a_1] ... Q_n[a_n] c_n, gauge-invariant) to <= 1e-10, in both tail modes;
  * the physics pins of tests/test_ptgen.py, now through the GPU generator AND the HIP propagation: the
    closed-form independent-boson coherence and the exact shift-register PT (oracle/ptgen_oracle.py)."""
import os

import numpy as np
import pytest

from oracle import oracle, ptgen_oracle
from pyaceqd_amd import engine, ptgen
from pyaceqd_amd.engine import Grid, System, Trajectories
from tests import helpers as H

pytestmark = pytest.mark.gpu
QDJ = lambda w: ptgen.qd_phonon_J(w, ae=3.0)  # noqa: E731


def _torch():
    import torch
    return torch


def _dev(a):
    torch = _torch()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.complex128, device="cuda")


def _rand(rng, m, n, rank=None, scale=None):
    A = rng.normal(size=(m, n)) + 1j * rng.normal(size=(m, n))
    if rank is not None:
        A = (rng.normal(size=(m, rank)) + 1j * rng.normal(size=(m, rank))) @ (
            rng.normal(size=(rank, n)) + 1j * rng.normal(size=(rank, n)))
        A += 1e-14 * (rng.normal(size=(m, n)) + 1j * rng.normal(size=(m, n)))
    if scale is not None:
        A = A * scale[None, :]
    return A


@pytest.mark.parametrize("small", ["1", "0"])
@pytest.mark.parametrize("m,n", [(7, 5), (5, 7), (195, 39), (40, 30), (300, 120), (930, 369), (600, 13), (100, 80),
                                 (64, 128)])
def test_ptg_qr_matches_lapack(monkeypatch, small, m, n):
    from pyaceqd_amd import ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", small)
    rng = np.random.default_rng(m * 1000 + n)
    W = _rand(rng, m, n)
    Qc, Rc, perm, k = ptgen_gpu.qr_cols(_dev(W.T))
    Q, R = Qc.T.cpu().numpy(), Rc.T.cpu().numpy()
    assert k == min(m, n) and np.array_equal(perm.cpu().numpy(), np.arange(n))
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(k))) < 1e-13
    assert np.max(np.abs(Q @ R - W)) < 1e-13 * np.max(np.abs(W)) * np.sqrt(m)
    assert np.max(np.abs(np.tril(R, -1))) == 0.0
    Rn = np.linalg.qr(W, mode="r")           # zgeqrf: the same Householder convention, real diagonal
    assert np.max(np.abs(R - Rn)) < 1e-12 * np.max(np.abs(Rn))


@pytest.mark.parametrize("mode", ["wg", "wg_blocked", "wave", "wave_qf"])
@pytest.mark.parametrize("m,n,kind", [(300, 120, "rand"), (930, 369, "rand"), (2955, 636, "graded"), (640, 273, "rand"),
                                      (500, 97, "lowrank"), (200, 200, "graded"), (129, 65, "rand"), (5000, 70, "rand")])
def test_ptg_qr_paths_match_lapack(monkeypatch, mode, m, n, kind):
    """plain QR on the multi-workgroup path, every kernel combination: workgroup-per-column step kernels (columns in
    registers; m > 4096 falls back to the per-wave kernels), the blocked factorization (panels of 32, trailing update
    V T^H V^H A), the per-wave kernels, and Q from blocks of 32 reflectors (default) or the per-wave Q kernel. Q
    orthonormal, W = Q R, R equal to LAPACK's (same reflectors), on random, graded (1 .. 1e-13) and numerically
    low-rank blocks"""
    from pyaceqd_amd import ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", "0")
    monkeypatch.setenv("PQD_PTG_WG", "0" if mode.startswith("wave") else "1")
    monkeypatch.setenv("PQD_PTG_BLOCKED", "1" if mode == "wg_blocked" else "0" if mode == "wg" else "-1")
    monkeypatch.setenv("PQD_PTG_QFB", "0" if mode == "wave_qf" else "1")
    rng = np.random.default_rng(m * 3 + n)
    if kind == "lowrank":
        W = _rand(rng, m, n, rank=n // 4)
    elif kind == "graded":
        W = _rand(rng, m, n, scale=np.logspace(0, -13, n))
    else:
        W = _rand(rng, m, n)
    Qc, Rc, perm, k = ptgen_gpu.qr_cols(_dev(W.T))
    Q, R = Qc.T.cpu().numpy(), Rc.T.cpu().numpy()
    assert k == n and np.array_equal(perm.cpu().numpy(), np.arange(n))
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(k))) < 1e-13
    assert np.max(np.abs(Q @ R - W)) < 1e-13 * np.max(np.abs(W)) * np.sqrt(m)
    assert np.max(np.abs(np.tril(R, -1))) == 0.0
    Rn = np.linalg.qr(W, mode="r")
    assert np.max(np.abs(R - Rn)) < 1e-12 * np.max(np.abs(Rn))


@pytest.mark.parametrize("wg", ["1", "0"])
@pytest.mark.parametrize("m,n,rank", [(1205, 300, 120), (400, 250, None), (5000, 90, 40)])
def test_ptg_qrcp_step_kernels(monkeypatch, wg, m, n, rank):
    """the rank-revealing pivoted QR on the workgroup-per-column and the per-wave step kernels: the same pivots
    and rank, Q orthonormal, W P = Q R + E within the tolerance"""
    from pyaceqd_amd import ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", "0")
    monkeypatch.setenv("PQD_PTG_WG", wg)
    rng = np.random.default_rng(m + 7 * n)
    W = _rand(rng, m, n, rank=rank, scale=None if rank else np.logspace(0, -14, n))
    tol = 1e-10 * np.max(np.linalg.norm(W, axis=0))
    Qc, Rc, perm, k = ptgen_gpu.qr_cols(_dev(W.T), pivot=True, tol=tol)
    Q, R, p = Qc.T.cpu().numpy(), Rc.T.cpu().numpy(), perm.cpu().numpy()
    assert sorted(p) == list(range(n))
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(k))) < 1e-12
    assert np.linalg.norm(W[:, p] - Q @ R) <= np.sqrt(n - k + 1) * tol * 1.01 + 1e-13 * np.linalg.norm(W)
    if rank is not None:
        assert k == rank
    monkeypatch.setenv("PQD_PTG_WG", "0" if wg == "1" else "1")
    _, _, perm2, k2 = ptgen_gpu.qr_cols(_dev(W.T), pivot=True, tol=tol)
    assert k2 == k and np.array_equal(perm2.cpu().numpy()[:k], p[:k])


@pytest.mark.parametrize("m,n,rank,tolmode", [(1205, 300, 120, "abs"), (400, 250, None, "abs"), (3000, 200, None, "rel"),
                                              (257, 64, 30, "rel"), (900, 40, None, "zero"), (150, 150, None, "abs"),
                                              (200, 70, 0, "abs"), (4096, 100, 60, "rel")])
def test_ptg_qrcp_persistent_equals_step_launches(monkeypatch, m, n, rank, tolmode):
    """the persistent pivoted QR (one launch, a grid barrier per step, csrc/ptgen.hip qrcp_persist_kernel) against one
    launch per step (PQD_PTG_QPERSIST=0): the same arithmetic, so Q, R, the pivots and the rank are equal bit for bit;
    with one poll per barrier wait (PQD_PTG_QSPIN=1) the barrier times out, the factorization is rerun from the saved
    copy (pqd_ptg_qr_counters counts it) and the results are still equal"""
    import ctypes
    from pyaceqd_amd import _lib, ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", "0")
    rng = np.random.default_rng(m + 3 * n)
    if rank == 0:
        W = np.zeros((m, n), complex)
    else:
        W = _rand(rng, m, n, rank=rank, scale=None if rank else np.logspace(0, -14, n))
    tol = {"abs": 1e-10 * np.max(np.linalg.norm(W, axis=0)), "rel": -1e-10, "zero": 0.0}[tolmode]
    dW = _dev(W.T)                                 # the device (torch's HIP runtime) before the library's first call
    out = {}
    for mode in ("step", "persist", "timeout"):
        monkeypatch.setenv("PQD_PTG_QPERSIST", "0" if mode == "step" else "1")
        monkeypatch.setenv("PQD_PTG_QSPIN", "1" if mode == "timeout" else str(1 << 22))
        fb0, fb1 = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(_lib.lib().pqd_ptg_qr_counters(ctypes.byref(fb0)))
        Qc, Rc, perm, k = ptgen_gpu.qr_cols(dW, pivot=True, tol=tol, unperm=tolmode == "rel")
        _lib.check(_lib.lib().pqd_ptg_qr_counters(ctypes.byref(fb1)))
        out[mode] = (Qc.cpu().numpy(), Rc.cpu().numpy(), perm.cpu().numpy(), k)
        if mode == "timeout" and rank != 0:       # (a zero matrix stops at step 0, before the first barrier)
            assert fb1.value > fb0.value          # n >= 40 workgroups: one poll cannot see them all arrive
        elif mode != "timeout":
            assert fb1.value == fb0.value
    for mode in ("persist", "timeout"):
        a, b = out["step"], out[mode]
        assert a[3] == b[3] and np.array_equal(a[2], b[2])
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    Q, R, p, k = out["persist"][0].T, out["persist"][1].T, out["persist"][2], out["persist"][3]
    if rank is not None:
        assert k == rank
    if k:
        assert np.max(np.abs(Q.conj().T @ Q - np.eye(k))) < 1e-12
        Wp = W if tolmode == "rel" else W[:, p]
        assert np.linalg.norm(Wp - Q @ R) <= 1e-9 * max(np.linalg.norm(W), 1e-300)


@pytest.mark.parametrize("m,n", [(2048, 128), (1205, 300), (400, 250), (3000, 200), (257, 64), (4096, 100), (150, 150),
                                 (100, 180)])
def test_ptg_qr_persistent_plain_equals_step_launches(monkeypatch, m, n):
    """plain Householder QR on the persistent kernel (PQD_PTG_QPERSIST=2) against one launch per reflector
    (PQD_PTG_PAIR=0, PQD_PTG_BLOCKED=0): equal bit for bit, also after a forced barrier timeout; and against LAPACK's R"""
    import ctypes
    from pyaceqd_amd import _lib, ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", "0")
    rng = np.random.default_rng(m + 5 * n)
    W = _rand(rng, m, n, scale=np.logspace(0, -12, n))
    dW = _dev(W.T)
    out = {}
    for mode in ("step", "persist", "timeout"):
        monkeypatch.setenv("PQD_PTG_QPERSIST", "0" if mode == "step" else "2")
        monkeypatch.setenv("PQD_PTG_PAIR", "0")
        monkeypatch.setenv("PQD_PTG_BLOCKED", "0")
        monkeypatch.setenv("PQD_PTG_QSPIN", "1" if mode == "timeout" else str(1 << 22))
        fb0, fb1 = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(_lib.lib().pqd_ptg_qr_counters(ctypes.byref(fb0)))
        Qc, Rc, perm, k = ptgen_gpu.qr_cols(dW)
        _lib.check(_lib.lib().pqd_ptg_qr_counters(ctypes.byref(fb1)))
        out[mode] = (Qc.cpu().numpy(), Rc.cpu().numpy(), k)
        assert (fb1.value > fb0.value) == (mode == "timeout")
    for mode in ("persist", "timeout"):
        assert out[mode][2] == out["step"][2] == min(m, n)
        assert np.array_equal(out[mode][0], out["step"][0]) and np.array_equal(out[mode][1], out["step"][1])
    Q, R = out["persist"][0].T, out["persist"][1].T
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(min(m, n)))) < 1e-13
    Rn = np.linalg.qr(W, mode="r")
    assert np.max(np.abs(R - Rn)) < 1e-12 * np.max(np.abs(Rn))


@pytest.mark.parametrize("small", ["1", "0"])
@pytest.mark.parametrize("m,n,rank", [(80, 39, 13), (60, 40, None), (1205, 300, 120), (400, 250, None), (700, 11, 5),
                                      (150, 50, None)])
def test_ptg_qrcp_rank_revealing(monkeypatch, small, m, n, rank):
    """column-pivoted QR stopping at a norm tolerance: Q orthonormal, pivots non-increasing, W P = Q R + E with
    ||E||_F <= sqrt(n - k) tol, and for a numerically rank-r matrix the rank found is r"""
    from pyaceqd_amd import ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", small)
    rng = np.random.default_rng(m + n)
    W = _rand(rng, m, n, rank=rank, scale=None if rank else np.logspace(0, -14, n))
    tol = 1e-10 * np.max(np.linalg.norm(W, axis=0))
    Qc, Rc, perm, k = ptgen_gpu.qr_cols(_dev(W.T), pivot=True, tol=tol)
    Q, R, p = Qc.T.cpu().numpy(), Rc.T.cpu().numpy(), perm.cpu().numpy()
    assert sorted(p) == list(range(n))
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(k))) < 1e-12
    E = W[:, p] - Q @ R
    assert np.linalg.norm(E) <= np.sqrt(n - k + 1) * tol * 1.01 + 1e-13 * np.linalg.norm(W)
    d = np.abs(np.diag(R[:, :k]))
    assert np.all(d[1:] <= d[:-1] * (1 + 1e-12))
    if rank is not None:
        assert k == rank
    # pivot = 2 (unperm): R in W's own column order, relative tolerance found on the device
    Qc2, Rc2, perm2, k2 = ptgen_gpu.qr_cols(_dev(W.T), pivot=True, tol=-1e-10, unperm=True)
    Q2, R2 = Qc2.T.cpu().numpy(), Rc2.T.cpu().numpy()
    assert k2 == k and np.array_equal(perm2.cpu().numpy(), p)
    assert np.max(np.abs(R2[:, p] - R)) == 0.0 and np.max(np.abs(Q2 - Q)) == 0.0
    assert np.linalg.norm(W - Q2 @ R2) <= np.sqrt(n - k + 1) * tol * 1.01 + 1e-13 * np.linalg.norm(W)


@pytest.mark.parametrize("small", ["1", "0", "0-persist", "0-rounds", "0-timeout"])
@pytest.mark.parametrize("r,c,graded", [(6, 9, False), (40, 200, True), (384, 1350, False), (300, 90, True),
                                         (120, 120, True), (45, 101, "lowrank"), (201, 700, "lowrank"),
                                         (1100, 700, True)])
def test_ptg_svd_matches_lapack(monkeypatch, small, r, c, graded):
    """thin SVD vs LAPACK on random, graded (1 .. 1e-13) and numerically low-rank blocks (odd sizes: the Jacobi
    tournament's dummy player; rank 1/4: three quarters of the columns at the rounding floor, as the stacked
    generator blocks are). Jacobi on the single-workgroup kernel, the persistent block kernel (two 4-column blocks per
    workgroup, n <= 512, default), the persistent column-pair kernel ("0-persist", n <= 1024), one launch per round
    ("0-rounds", also what n > 1024 uses), and a persistent launch whose grid barrier times out and is rerun per round
    from a copy of X ("0-timeout")"""
    from pyaceqd_amd import ptgen_gpu
    monkeypatch.setenv("PQD_PTG_SMALL", small[0])
    monkeypatch.setenv("PQD_PTG_JPERSIST", "0" if small == "0-rounds" else "1")
    monkeypatch.setenv("PQD_PTG_JBLOCK", "0" if small in ("0-rounds", "0-persist") else "1")
    # 0-timeout: one poll per barrier wait, so the persistent launch times out and is rerun per round from a copy
    monkeypatch.setenv("PQD_PTG_JSPIN", "1" if small == "0-timeout" else str(1 << 22))
    rng = np.random.default_rng(r * 7 + c)
    k = min(r, c)
    if graded == "lowrank":
        A = _rand(rng, r, c, rank=k // 4)
    elif graded:
        U0 = np.linalg.qr(_rand(rng, r, k))[0]
        V0 = np.linalg.qr(_rand(rng, c, k))[0]
        A = (U0 * np.logspace(0, -13, k)[None, :]) @ V0.conj().T
    else:
        A = _rand(rng, r, c)
    import ctypes
    from pyaceqd_amd import _lib
    dA = _dev(A)                                   # the device (torch's HIP runtime) before the library's first call
    fb0 = ctypes.c_int32(0)
    _lib.check(_lib.lib().pqd_ptg_counters(ctypes.byref(fb0)))
    U, S, Vh = (x.cpu().numpy() for x in ptgen_gpu.svd(dA))
    fb1 = ctypes.c_int32(0)
    _lib.check(_lib.lib().pqd_ptg_counters(ctypes.byref(fb1)))
    if small == "0-timeout" and min(r, c) >= 64:  # several workgroups: the fallback ran
        assert fb1.value > fb0.value
    elif small != "0-timeout":
        assert fb1.value == fb0.value
    Sn = np.linalg.svd(A, compute_uv=False)
    kk = len(S)                                    # the numerical rank at 1e-14 (the rest is dropped)
    assert np.max(np.abs(S - Sn[:kk])) < 1e-13 * Sn[0]
    assert np.all(Sn[kk:] < 1e-12 * Sn[0])
    assert np.all(np.diff(S) <= 0)
    # singular vectors of the numerical rank (the null space of a rank-deficient block is arbitrary: its columns sit at
    # the rounding floor and are never rotated, and the generator truncates them away)
    kr = min(kk, int(np.count_nonzero(Sn > 1e-13 * Sn[0])))
    assert np.max(np.abs(U[:, :kr].conj().T @ U[:, :kr] - np.eye(kr))) < 1e-12
    assert np.max(np.abs(Vh[:kr] @ Vh[:kr].conj().T - np.eye(kr))) < 1e-12
    assert np.max(np.abs((U * S[None, :]) @ Vh - A)) < 1e-13 * Sn[0] * np.sqrt(max(r, c))


@pytest.mark.parametrize("scale", [1e-150, 1e81, 1e150])
def test_ptg_svd_extreme_scale(scale):
    """the generator's boundary blocks reach 1e81 and beyond (the future-influence MPS norm grows like sqrt(P)^K):
    the device SVD scales internally, so squared column norms and the Jacobi test never overflow (found on the
    K = 205 biexciton PT, where the unscaled Jacobi did not converge)"""
    from pyaceqd_amd import ptgen_gpu
    rng = np.random.default_rng(5)
    A0 = _rand(rng, 384, 700, scale=np.logspace(0, -11, 700))
    U, S, Vh = (x.cpu().numpy() for x in ptgen_gpu.svd(_dev(A0 * scale)))
    Sn = np.linalg.svd(A0, compute_uv=False)
    assert np.max(np.abs(S / scale - Sn[:len(S)])) < 1e-13 * Sn[0]
    assert np.max(np.abs((U * (S / scale)[None, :]) @ Vh - A0)) < 1e-13 * Sn[0] * np.sqrt(700)


# ---------------------------------------------------------------------------------------------------- the PT
def influence(pt, paths):
    """bond0 Q_s(1)[g(a_1)] ... Q_s(n)[g(a_n)] c_s(n) for each path of Liouville indices (the slice schedule of
    engine semantics: slice n for n < n_init, then the repeated slices)"""
    out = []
    for path in paths:
        v = pt.bond0.copy()
        s = 0
        for n, a in enumerate(path):
            s = n if n < pt.n_init else pt.n_init + (n - pt.n_init) % (pt.n_slices - pt.n_init)
            v = v @ pt.Q[s, pt.gmap[a]]
        out.append(v @ pt.closure[s])
    return np.array(out)


@pytest.mark.parametrize("tail", ["svd", "qrcp"])
@pytest.mark.parametrize("lam,K,T,mb", [([0, 1, 1, 2], 4, 4.0, 0), ([0, 1], 5, 4.0, 0), ([0, 1, 1, 2, 2, 3], 3, 1.0, 0),
                                        ([0, 1, 1, 2], 6, 4.0, 32)])
def test_gpu_generator_matches_host_influence(tail, lam, K, T, mb):
    """GPU generator vs ptgen.py (the host restatement) on the same parameters: influence values of 400 random
    paths spanning the explicit and the repeated slices agree to 1e-10 (threshold 1e-11; bond uncapped (chi 54-132),
    and capped at 32 where the cap, not the threshold, decides the slice: the same top-32 subspace)"""
    from pyaceqd_amd import ptgen_gpu
    A = np.diag(np.array(lam, dtype=float))
    eta, delta = ptgen.eta_coefficients(QDJ, T, 0.1, K)
    ph = ptgen.build_gaussian_pt(A, 0.1, eta, delta, threshold=1e-11, max_bond=mb)
    pg = ptgen_gpu.build_gaussian_pt_gpu(A, 0.1, eta, delta, threshold=1e-11, max_bond=mb, tail=tail)
    assert pg.n_init == ph.n_init == 2 * K and pg.n_slices == ph.n_slices
    rng = np.random.default_rng(K + len(lam))
    N2 = len(lam) ** 2
    paths = [rng.integers(0, N2, size=rng.integers(1, 3 * K + 4)) for _ in range(400)]
    a, b = influence(pg, paths), influence(ph, paths)
    assert np.max(np.abs(a - b)) < 1e-10 * np.max(np.abs(b))
    assert np.max(np.abs(b)) > 0.1


@pytest.mark.parametrize("lam,K,n_init", [([0, 1], 3, 9), ([0, 1, 1], 2, 4), ([0, 1, 1, 2], 2, 7), ([0, 2], 1, 2)])
def test_gpu_generator_exact_shift_register_on_hip(lam, K, n_init):
    """test_ptgen.py's shift-register pin through the GPU generator, propagated on the HIP sweep: driven, damped
    N-level system, 30x bath, threshold 1e-14, 40 steps vs the exact uncompressed PT (oracle/ptgen_oracle.py)"""
    from pyaceqd_amd import ptgen_gpu
    N = len(lam)
    A = np.diag(np.array(lam, dtype=float))
    J = lambda w: 30 * QDJ(w)  # noqa: E731
    eta, delta = ptgen.eta_coefficients(J, 4.0, 0.1, K)
    sysd, grid = H.random_system(N, n_steps=40, seed=3 + N)
    rho0 = H.random_rho(N)
    ops = [H.ketbra(N, i, j) for i in range(N) for j in range(N)]
    tr = Trajectories(np.array([0, 5]), np.array([40, 33]))
    pg = ptgen_gpu.build_gaussian_pt_gpu(A, 0.1, eta, delta, threshold=1e-14, max_bond=0, n_init=n_init)
    pe = ptgen_oracle.exact_if_pt(A, eta, delta, 0.1)
    got = engine.propagate(sysd, grid, rho0, ops, tr, pt=pg)
    ref = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pe)
    bare = oracle.propagate(sysd, grid, rho0, ops, tr)
    for a, b, c in zip(got, ref, bare):
        assert np.max(np.abs(a - b)) < 1e-11
        assert np.max(np.abs(b - c)) > 1e-2


@pytest.mark.parametrize("K,thr", [(4, 1e-10), (5, 1e-11)])
def test_gpu_generator_ibm_on_hip(K, thr):
    """undriven pure dephasing of a TLS with QD phonons at 4 K (8K steps: explicit, then repeated slices) through
    the GPU generator AND the HIP sweep vs the discretised independent-boson coherence: <= 1e-6 relative at every
    step (the north star's phonon tolerance; the host generator reaches 4e-9 / 5e-10 here, chi 49 / 110), trace
    preserved"""
    from pyaceqd_amd import ptgen_gpu
    dt = 0.1
    eta, delta = ptgen.eta_coefficients(QDJ, 4.0, dt, K)
    pt = ptgen_gpu.build_gaussian_pt_gpu(np.diag([0.0, 1.0]), dt, eta, delta, threshold=thr, max_bond=0)
    assert pt.chi <= 128
    n = 8 * K
    out = engine.propagate(System(dim=2, H0=np.zeros((2, 2))), Grid(0.0, dt, n), 0.5 * np.ones((2, 2), complex),
                           [H.ketbra(2, 0, 1), np.eye(2)], Trajectories(np.array([0]), np.array([n])), pt=pt)[0]
    ex = ptgen_oracle.ibm_coherence_discrete(eta, delta, dt, n)
    assert np.max(np.abs(out[:, 0] - ex) / np.abs(ex)) < 1e-6
    assert np.max(np.abs(out[:, 1] - 1)) < 1e-9


def test_driver_generates_on_the_gpu(tmp_path, monkeypatch):
    """system_ace_stream(phonons=True) without a PT file generates the PT on the GPU by default; the cached PT has
    the host generator's influence values (PQD_PTGEN=host)"""
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd import opgrammar
    B = opgrammar.to_matrix("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4", 4)
    kw = dict(dt=0.1, t_mem=0.4, ae=3.0, temperature=4, threshold="11", factor_ah=None, boson_e_max=7, J_file=None,
              J_to_file=None, use_infinite=False, system_prefix="bx", temp_dir=str(tmp_path) + os.sep, verbose=False)
    called = []
    from pyaceqd_amd import ptgen_gpu
    real = ptgen_gpu.qd_phonon_pt_gpu
    monkeypatch.setattr(ptgen_gpu, "qd_phonon_pt_gpu", lambda *a, **k: called.append(1) or real(*a, **k))
    pg = gs._resolve_pt(None, B, **kw)
    assert called
    monkeypatch.setenv("PQD_PTGEN", "host")
    ph = gs._resolve_pt(None, B, **dict(kw, temp_dir=str(tmp_path / "h") + os.sep))
    rng = np.random.default_rng(1)
    paths = [rng.integers(0, 16, size=rng.integers(1, 14)) for _ in range(200)]
    a, b = influence(pg, paths), influence(ph, paths)
    assert np.max(np.abs(a - b)) < 1e-10 * np.max(np.abs(b))


def test_gpu_generator_biexciton_reference_default_timed():
    """the biexciton PT at the reference's own defaults (four_level_system/linear.py:8: dt 0.5, t_mem 20.48 ->
    K = 41, T 4 K, threshold 1e-10, bond cap 128): generated on the GPU in well under a minute, slices bounded,
    trace preserving (closure of the trace path = 1 for every step of a free run)"""
    import time
    from pyaceqd_amd import ptgen_gpu
    t0 = time.perf_counter()
    pt = ptgen_gpu.qd_phonon_pt_gpu(np.diag([0.0, 1.0, 1.0, 2.0]), 0.5, t_mem=20.48, ae=3.0, temperature=4,
                                    threshold=1e-10)
    el = time.perf_counter() - t0
    print(f"biexciton K=41 PT on the GPU: {el:.1f} s, chi {pt.chi}, slices {pt.n_slices}")
    assert pt.n_init == 82 and pt.chi <= 128
    assert el < 60.0
    # the path that stays on |0><0| (coupling eigenvalue 0 on both sides) has influence exactly 1; the PT keeps it to
    # its truncation error (the bond cap of 128 binds here; measured 1.2e-7 after 120 steps)
    inf = influence(pt, [np.zeros(n, dtype=int) for n in (1, 10, 82, 120)])
    assert np.max(np.abs(inf - 1)) < 1e-6


# ---------------------------------------------------- use_infinite at the tls defaults
def test_tls_reference_default_phonons_ibm_on_hip(tmp_path):
    """tls(phonons=True) at the reference's own defaults (tls.py:16-18: dt 0.1, a_e 5 nm, 4 K, threshold 8,
    use_infinite=True) through the drop-in driver: the PT generated on the GPU with the bath's own memory (K = 65 of
    the te = 12.8 ps horizon, converged), propagated on the HIP sweep, an undriven dot from (|0> + |1>)/sqrt 2
    against the closed-form independent-boson coherence (continuous integral, independent quadrature) for 40 ps.
    The bound is the generator's own accuracy at threshold 1e-8 (measured 6.1e-4 relative after 400 steps with the
    host generator; 3.2e-5 at threshold 1e-10: the bond truncation, not the memory, sets it)."""
    from pyaceqd_amd.two_level_system.tls import tls
    t_end = 40.0
    res = tls(0, t_end, phonons=True, rho0=0.5 * np.ones((2, 2), complex), output_ops=["|0><1|_2", "|0><0|_2"],
              temp_dir=str(tmp_path) + os.sep)
    from pyaceqd_amd.pt import load_pt
    f = [x for x in os.listdir(tmp_path) if x.endswith(".pt.npz")]
    assert len(f) == 1
    meta = load_pt(str(tmp_path / f[0])).meta
    assert meta["infinite"] and meta["converged"] and meta["K"] == 65 and meta["generator"] == "gpu"
    J = lambda w: ptgen.qd_phonon_J(w, ae=5.0)  # noqa: E731
    t = np.real(res[0])
    ex = ptgen_oracle.ibm_coherence_exact(J, 4.0, t)
    err = np.abs(res[1] - ex) / np.abs(ex)
    print(f"tls default phonons: max rel err {err.max():.2e} (at {t[np.argmax(err)]:.1f} ps), K {meta['K']}")
    assert np.max(err) < 1.5e-3
    assert np.max(np.abs(res[2] - 0.5)) < 1e-9          # populations do not move in the IBM


def test_gpu_infinite_memory_pt_converged_at_tls_default():
    """the memory the use_infinite rule picks at the tls defaults (K = 65 for threshold 1e-8) is converged: with the
    compression made finer (threshold 1e-9, so its own noise does not mask the memory), doubling the memory (K = 130)
    moves the influence values of 200 random paths over the explicit slices (<= 140 steps) by <= 10 x 1e-8 (measured
    1.8e-8 with the host generator), while at the default compression the same comparison moves them by ~1.7e-7,
    no more than another compression of the same memory does (threshold 1e-8 vs 1e-9: ~2e-7): the PT's error at the
    defaults is the compression's, not the memory's"""
    from pyaceqd_amd import ptgen_gpu
    B = np.diag([0.0, 1.0])
    kw = dict(t_mem=6.4, ae=5.0, temperature=4, use_infinite=True)
    p1 = ptgen_gpu.qd_phonon_pt_gpu(B, 0.1, threshold=1e-8, **kw)
    assert p1.meta["K"] == 65 and p1.meta["converged"]
    f65 = ptgen_gpu.qd_phonon_pt_gpu(B, 0.1, threshold=1e-9, K=65, **kw)
    f130 = ptgen_gpu.qd_phonon_pt_gpu(B, 0.1, threshold=1e-9, K=130, **kw)
    p2 = ptgen_gpu.qd_phonon_pt_gpu(B, 0.1, threshold=1e-8, K=130, **kw)
    rng = np.random.default_rng(2)
    paths = [rng.integers(0, 4, size=rng.integers(1, 141)) for _ in range(200)]
    inf = {k: influence(p, paths) for k, p in (("d65", p1), ("d130", p2), ("f65", f65), ("f130", f130))}
    d = lambda a, b: float(np.max(np.abs(inf[a] - inf[b])) / np.max(np.abs(inf[b])))  # noqa: E731
    d_mem, d_mem_default, d_comp = d("f65", "f130"), d("d65", "d130"), d("d65", "f65")
    print(f"memory 65 vs 130 at compression 1e-9: {d_mem:.2e}; at 1e-8: {d_mem_default:.2e}; "
          f"compression 1e-8 vs 1e-9 at K 65: {d_comp:.2e}")
    assert d_mem <= 10 * 1e-8
    assert d_mem_default <= 2 * d_comp + 1e-8


def test_engine_refuses_pt_of_another_dt():
    """engine.propagate raises on a PT generated for another dt before anything is launched"""
    pt = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), 0.5, *ptgen.eta_coefficients(QDJ, 4.0, 0.5, 2), threshold=1e-8)
    with pytest.raises(ValueError, match="dt = 0.5"):
        engine.propagate(System(dim=2, H0=np.zeros((2, 2))), Grid(0.0, 0.1, 10), np.eye(2) / 2, [np.eye(2)],
                         Trajectories(np.array([0]), np.array([10])), pt=pt)


def test_ptg_scratch_per_stream_and_convergence_on_last_sweep():
    """factorizations queued on two streams at once use separate scratch (a plain QR returns with its
    kernels still queued), and a Jacobi that converges on its last allowed sweep is not reported as a failure"""
    from pyaceqd_amd import ptgen_gpu, _lib
    torch = _torch()
    rng = np.random.default_rng(11)
    A1, A2 = _rand(rng, 700, 300), _rand(rng, 500, 200)
    s1 = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        W1 = _dev(A1.T)
        Q1, R1, _, k1 = ptgen_gpu.qr_cols(W1)
    W2 = _dev(A2.T)
    Q2, R2, _, k2 = ptgen_gpu.qr_cols(W2)                 # default stream, while s1's kernels may still run
    torch.cuda.synchronize()
    for A, Q, R in ((A1, Q1, R1), (A2, Q2, R2)):
        Qh, Rh = Q.cpu().numpy().T, R.cpu().numpy().T
        assert np.max(np.abs(Qh @ Rh - A)) < 1e-12 * np.max(np.abs(A)) * 30
    X = _rand(rng, 96, 96)
    ptgen_gpu.jacobi_cols(_dev(X.T), max_sweeps=60)
    need = ptgen_gpu.LAST_SWEEPS
    assert 2 <= need < 60
    ptgen_gpu.jacobi_cols(_dev(X.T), max_sweeps=need)         # converges on its last allowed sweep
    assert ptgen_gpu.LAST_SWEEPS == need
    with pytest.raises(_lib.PQDError, match="no convergence"):
        ptgen_gpu.jacobi_cols(_dev(X.T), max_sweeps=need - 1)


def test_tls_threshold_1e10_uncapped_bond_beats_the_cap_ibm(monkeypatch):
    """at the tls phonon defaults (dt 0.1, a_e 5 nm, 4 K, K = 65 of the bath's own memory) a
    threshold of 1e-10 asks for bonds up to ~160, past the batched kernel's cap of 128. Generated on the GPU with the
    cap lifted to 256 (PQD_PT_MAX_BOND, the split groups' streamed-slice path), the cut is the threshold's (recorded:
    no cap-bound cut) and the undriven dot's coherence is closer to the closed-form independent-boson solution over
    40 ps than with the cap binding (host generator: 2.0e-5 against 3.0e-5 relative); at 1e-11 (bond ~200, still
    the threshold's cut) it falls to 2.2e-6: the error falls with the threshold once the cap no longer decides."""
    from pyaceqd_amd import ptgen_gpu
    dt, n = 0.1, 400
    J = lambda w: ptgen.qd_phonon_J(w, ae=5.0)  # noqa: E731
    eta, delta = ptgen.eta_coefficients(J, 4.0, dt, 65)
    t = dt * np.arange(n + 1)
    ex = ptgen_oracle.ibm_coherence_exact(J, 4.0, t)

    def run(thr, cap):
        pt = ptgen_gpu.build_gaussian_pt_gpu(np.diag([0.0, 1.0]), dt, eta, delta, threshold=thr, max_bond=cap)
        out = engine.propagate(System(dim=2, H0=np.zeros((2, 2))), Grid(0.0, dt, n), 0.5 * np.ones((2, 2), complex),
                               [H.ketbra(2, 0, 1), np.eye(2)], Trajectories(np.array([0]), np.array([n])), pt=pt)[0]
        assert np.max(np.abs(out[:, 1] - 1)) < 1e-9
        return pt, float(np.max(np.abs(out[:, 0] - ex) / np.abs(ex)))

    pt_free, e_free = run(1e-10, 256)
    tr = pt_free.meta["truncation"]
    assert pt_free.chi > 128 and not tr["cap_decided"] and tr["max_discarded_rel"] <= 1e-10
    with pytest.warns(RuntimeWarning, match="bond cap 128"):
        pt_cap, e_cap = run(1e-10, 128)
    assert pt_cap.meta["truncation"]["cap_decided"]
    pt_11, e_11 = run(1e-11, 256)
    print(f"tls 1e-10: chi {pt_free.chi} err {e_free:.2e}; capped at 128 {e_cap:.2e}; 1e-11: chi {pt_11.chi} "
          f"err {e_11:.2e}")
    assert e_free < 2.6e-5 < e_cap < 3.2e-5 * 1.2
    assert pt_11.chi > pt_free.chi and not pt_11.meta["truncation"]["cap_decided"] and e_11 < 5e-6
