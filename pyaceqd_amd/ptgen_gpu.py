"""Gaussian-bath PT generator on the GPU: the same construction as pyaceqd_amd/ptgen.py (the host restatement of
ACE's `dont_propagate` + `write_PT` step, reference general_system.py:152-211), with every factorization on the
device through libpqd's hand-written HIP kernels (csrc/ptgen.hip, C-ABI pqd_ptg_qr / pqd_ptg_jacobi) and the
tensors resident in HBM between steps.

Per PT step the host algorithm compresses a K-site "future influence" MPS twice (s+ half, s- half): a right-to-left
QR sweep (right-canonical form), the boundary SVD (its phase-fixed isometry is the PT slice) and a left-to-right
truncating sweep (ptgen._compress). Here:
  * QR sweep: Householder QR on the device (pqd_ptg_qr, pivot = 0);
  * boundary SVD: QR, then one-sided Jacobi on the R factor (pqd_ptg_jacobi): every singular value to high relative
    accuracy, so the threshold / bond-cap truncation and the phase fix (ptgen._fix_phase) are the host's;
  * truncating sweep: tail="svd" uses the same SVD (the host algorithm step for step); tail="qrcp" (default) uses a
    column-pivoted QR that stops at the threshold instead (a rank-revealing truncation whose discarded Frobenius
    norm is bounded like the SVD's, sqrt(n) * threshold * sigma_max). The tail's internal gauge and truncation do
    not enter the slices except through the tail function itself, so the two modes give the same PT to the
    threshold; the QRCP sweep is several times cheaper (no Jacobi sweeps on the tail blocks).
Contractions, stacking and reshapes are torch operations on the device (rocBLAS zgemm: plumbing).

The public entry points mirror ptgen's: GaussianPTBuilderGPU (step / closure / stationary_slice),
build_gaussian_pt_gpu, qd_phonon_pt_gpu. They return the same ProcessTensor (host numpy arrays)."""
import ctypes as C
import os
import time

import numpy as np

from . import _lib
from . import ptgen
from .engine import ProcessTensor


_DEBUG = bool(int(os.environ.get("PQD_PTG_DEBUG", "0") or 0))
# PQD_PTG_PHASES=1: wall time per compression phase (synchronising: diagnostics only, scripts/bench_ptgen.py)
_PHASES = {"rcanon": 0.0, "svd": 0.0, "lr": 0.0} if os.environ.get("PQD_PTG_PHASES") == "1" else None
_STATS = []  # (kind, sizes...) per factorization when PQD_PTG_DEBUG=1 (scripts/bench_ptgen.py --stats)
LAST_SWEEPS = 0  # sweeps of the last jacobi_cols call (tests)
RETRIES = []  # (n, attempt) of every boundary SVD whose Jacobi needed another attempt (svd below)


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.PQDError("the GPU PT generator needs a ROCm device (torch.cuda.is_available() is False)")
    return torch


def _stream(torch, dev=None):
    """the current stream of the tensor's device (the library keys its scratch by device and stream)"""
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def qr_cols(Wc, pivot=False, tol=0.0, unperm=False):
    """Householder QR of W (m x n) given as Wc (n, m): row j of Wc is column j of W (a column-major buffer).
    Returns (Qc (rank, m): row i = column i of Q, Rc (n, rank): row j = column j of R (pivoted order), perm (n,),
    rank). pivot: column pivoting with a stop at trailing column norm <= tol (absolute)."""
    torch = _torch()
    n, m = Wc.shape
    W = Wc.resolve_conj().resolve_neg().contiguous()  # a conj view / strided view is materialised here ...
    if W.data_ptr() == Wc.data_ptr():
        W = W.clone()                                 # ... else copy: W is overwritten
    kmax = min(m, n)
    Q = torch.empty(kmax * m, dtype=torch.complex128, device=W.device)
    R = torch.empty(max(kmax, 1) * n, dtype=torch.complex128, device=W.device)
    perm = torch.empty(n, dtype=torch.int32, device=W.device)
    rank = C.c_int32(0)
    with torch.cuda.device(W.device):   # the launches go to W's device, on that device's current stream
        _lib.check(_lib.lib().pqd_ptg_qr(_stream(torch, W.device), C.c_void_p(W.data_ptr()), int(m), int(n),
                                         (2 if unperm else 1) if pivot else 0,
                                         float(tol), C.c_void_p(Q.data_ptr()), C.c_void_p(R.data_ptr()),
                                         C.c_void_p(perm.data_ptr()), C.byref(rank)))
    k = rank.value
    if _DEBUG:
        _STATS.append(("qrcp" if pivot else "qr", m, n, k))
    return Q[: k * m].view(k, m), R[: k * n].view(n, k), (perm.long() if pivot else perm), k


def jacobi_cols(Xc, tol=None, max_sweeps=60, zero_tol=1e-16):
    """One-sided Jacobi SVD of the square X given as Xc (n, n) (row j = column j of X): X V = U diag(sigma).
    Returns (Uc (n, n): row j = unit column j of U, Vc (n, n): row j = column j of V, sigma (n,)), unsorted.
    tol (default max(16, n) eps): a pair is rotated while |x_p^H x_q| > tol |x_p| |x_q|. The computed inner product
    of two orthogonal columns carries a rounding error up to ~n eps |x_p| |x_q|, so a tighter tol never stops on
    rank-deficient blocks (whose tiny columns are rounding noise of the large ones); singular values stay accurate
    to ~tol relative. Columns below zero_tol ||X||_F are numerically zero and never rotated (their singular values
    come out as their norms, at the rounding floor)."""
    torch = _torch()
    n = Xc.shape[0]
    if tol is None:
        tol = max(16, n) * 2.220446049250313e-16
    X = Xc.resolve_conj().resolve_neg().contiguous()
    if X.data_ptr() == Xc.data_ptr():
        X = X.clone()
    V = torch.empty((n, n), dtype=torch.complex128, device=X.device)
    sig = torch.empty(n, dtype=torch.float64, device=X.device)
    sw = C.c_int32(0)
    with torch.cuda.device(X.device):
        _lib.check(_lib.lib().pqd_ptg_jacobi(_stream(torch, X.device), C.c_void_p(X.data_ptr()), int(n),
                                             C.c_void_p(V.data_ptr()), C.c_void_p(sig.data_ptr()), float(tol),
                                             float(zero_tol), int(max_sweeps), C.byref(sw)))
    global LAST_SWEEPS
    LAST_SWEEPS = sw.value
    if sw.value > max_sweeps:   # the library reports max_sweeps + 1 when the last allowed sweep still rotated
        raise _lib.PQDError(f"pqd_ptg_jacobi: no convergence in {max_sweeps} sweeps (n = {n})")
    if _DEBUG:
        _STATS.append(("jacobi", n, sw.value))
    return X, V, sig


_JZERO = float(os.environ.get("PQD_PTG_JZERO", "1e-16") or 1e-16)  # Jacobi zero-column threshold (A/B runs)
_JT = os.environ.get("PQD_PTG_JT", "1") == "1"                     # Jacobi on R2^H (DV), 0: on R2 (A/B runs)


def svd(A, rank_tol=1e-14):
    """Thin SVD of A (r x c, device complex128): (U (r, k), S (k,), Vh (k, c)), S descending, k = the numerical
    rank at rank_tol (directions below rank_tol x the largest column norm are dropped: far below any truncation
    threshold the generator uses).

    Preconditioned one-sided Jacobi (Drmac-Veselic): W (= A or A^H, whichever is tall) P = Q1 R1 by a rank-revealing
    column-pivoted QR; B = R1 P^T (k x n) is factored again, B^H = Q2 R2; the Jacobi sweeps run on the small square
    R2, whose columns are already nearly orthogonal, so they converge in a few sweeps. W = (Q1 V) S (Q2 Uhat)^H with
    R2 V = Uhat S."""
    torch = _torch()
    r, c = A.shape
    # scale to max |a_ij| = 1 (on the device, no host pass): the generator's boundary blocks reach 1e81 and more (the
    # future-influence MPS norm grows like sqrt(P)^K), where the Jacobi test |x_p^H x_q| > tol sqrt(|x_p|^2 |x_q|^2)
    # overflows; LAPACK scales the same way
    amax = torch.amax(A.abs())
    sc = torch.where(amax > 0, amax, torch.ones_like(amax))
    A = A / sc
    Wc = A.conj() if r <= c else A.T             # rows of Wc = columns of W (tall: m = max(r, c), n = min(r, c))
    n, m = Wc.shape
    Q1c, R1c, perm, k1 = qr_cols(Wc, pivot=True, tol=-rank_tol, unperm=True)  # rank_tol x the largest column norm
    if k1 == 0:                                    # a zero block: one zero singular value
        U = torch.zeros((r, 1), dtype=A.dtype, device=A.device)
        Vh = torch.zeros((1, c), dtype=A.dtype, device=A.device)
        U[0, 0] = Vh[0, 0] = 1.0
        return U, torch.zeros(1, dtype=torch.float64, device=A.device), Vh
    B = R1c.T                                      # R1 P^T (k1 x n)
    Q2c, R2c, _, k2 = qr_cols(B.conj())          # B^H = Q2 R2 (n x k1, k1 x k1)
    attempts = [(_JT, _JZERO), (not _JT, _JZERO), (_JT, max(_JZERO, 1e-13))]
    for ia, (jt, zt) in enumerate(attempts):
        # the two orientations give the same SVD; R2^H (Drmac-Veselic) usually needs fewer sweeps (8 against 10 on
        # the biexciton boundary blocks). A block on which one does not converge is tried on the other, then with
        # columns below 1e-13 ||X||_F left unrotated (far below any truncation threshold the generator uses)
        try:
            if jt:                                 # Jacobi on X = R2^H: X V = Uhat S, W = (Q1 Uhat) S (Q2 V)^H
                Xc, Vc, sig = jacobi_cols(R2c.conj().T, zero_tol=zt)
                o = torch.argsort(sig, descending=True, stable=True)
                UW = (Xc[o] @ Q1c).T
                VhW = (Vc[o] @ Q2c).conj()
            else:                                  # Jacobi on R2: R2 V = Uhat S, W = (Q1 V) S (Q2 Uhat)^H
                Xc, Vc, sig = jacobi_cols(R2c, zero_tol=zt)
                o = torch.argsort(sig, descending=True, stable=True)
                UW = (Vc[o] @ Q1c).T               # (m, k1): columns Q1 v_o
                VhW = (Xc[o] @ Q2c).conj()         # (k1, n): rows (Q2 uhat_o)^H
            break
        except _lib.PQDError as e:
            if "no convergence" not in str(e) or ia == len(attempts) - 1:
                if os.environ.get("PQD_PTG_DUMP"):     # the block, for offline analysis
                    np.save(os.environ["PQD_PTG_DUMP"], R2c.cpu().numpy())
                raise
            RETRIES.append((int(R2c.shape[0]), ia))
    S = sig[o] * sc
    if r <= c:                                     # W = A^H
        return VhW.conj().T, S, UW.conj().T
    return UW, S, VhW


def _keep(S_host, threshold, max_k):
    return ptgen._keep(S_host, threshold, max_k)


def _fix_phase(U, Vh):
    """ptgen._fix_phase on the device (largest-|.| entry of every left singular vector real positive)"""
    torch = _torch()
    idx = torch.argmax(U.abs(), dim=0)
    ph = U[idx, torch.arange(U.shape[1], device=U.device)]
    ph = ph / torch.clamp(ph.abs(), min=1e-300)
    return U * ph.conj()[None, :], Vh * ph[:, None]


def _rcanon(mps):
    """ptgen._rcanon on the device: right-canonical QR sweep over sites len-1 .. 1"""
    torch = _torch()
    for j in range(len(mps) - 1, 0, -1):
        T = mps[j]
        cl, P, cr = T.shape
        # T = R^H Q^H from the QR of T^H; Householder QR commutes with conjugation (zlarfg: beta real, tau and v
        # conjugate), so the QR of T^T = conj(T^H) hands over conj(Q), conj(R) without materialising T^H
        Qc, Rc, _, k = qr_cols(T.reshape(cl, P * cr))
        mps[j] = Qc.reshape(k, P, cr)
        mps[j - 1] = torch.tensordot(mps[j - 1], Rc, dims=([2], [0]))


def _compress(mps, threshold, max_bond, tail_threshold=None, tail_max_bond=None, tail="qrcp", stats=None):
    """ptgen._compress on the device. Returns (U, mps') with U the phase-fixed isometry of the boundary SVD; `stats`
    (ptgen.TruncationStats) records what decided the boundary cut."""
    torch = _torch()
    tthr = threshold if tail_threshold is None else tail_threshold
    tm = _PHASES is not None
    if tm:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    _rcanon(mps)
    if tm:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    T = mps[0]
    L, P, cr = T.shape
    U, S, Vh = svd(T.reshape(L, P * cr))
    if tm:
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    Sh = S.cpu().numpy()
    k = _keep(Sh, threshold, max_bond)
    if stats is not None:
        stats.record(Sh, k)
    U, Vh = _fix_phase(U[:, :k], Vh[:k])
    cur = (S[:k, None].to(Vh.dtype) * Vh).reshape(k, P, cr)
    for j in range(len(mps) - 1):
        cl, P, cr = cur.shape
        M = cur.reshape(cl * P, cr)
        if tail == "svd":
            u, s, vh = svd(M)
            kk = _keep(s.cpu().numpy(), tthr, tail_max_bond)
            mps[j] = u[:, :kk].reshape(cl, P, kk)
            carry = s[:kk, None].to(vh.dtype) * vh[:kk]
        else:
            Qc, Rc, perm, kk = qr_cols(M.T, pivot=True, tol=-tthr, unperm=True)  # tthr x the largest column norm
            if kk == 0:                            # M == 0: keep one (zero-weight) bond direction
                kk = 1
                Qc = torch.zeros((1, M.shape[0]), dtype=M.dtype, device=M.device)
                Qc[0, 0] = 1.0
                Rc = torch.zeros((M.shape[1], 1), dtype=M.dtype, device=M.device)
            if tail_max_bond and kk > tail_max_bond:
                kk = tail_max_bond
                Qc, Rc = Qc[:kk], Rc[:, :kk]
            mps[j] = Qc.T.reshape(cl, P, kk)
            carry = Rc.T                           # R P^T
        cur = torch.tensordot(carry, mps[j + 1], dims=([1], [0]))
    mps[-1] = cur
    if tm:
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        _PHASES["rcanon"] += t1 - t0
        _PHASES["svd"] += t2 - t1
        _PHASES["lr"] += t3 - t2
    return U, mps


def _stack(first, later, F, new):
    """ptgen._stack on the device (block-diagonal direct sum over beta)"""
    torch = _torch()
    nb = first.shape[0]
    chain = [first] + [torch.einsum("bpq,lqr->blpr", F[:, j], T) for j, T in enumerate(later)]
    if new is not None:
        chain.append(new[:, None, :, None])
    out = []
    ar = torch.arange(nb, device=first.device)
    for j, blk in enumerate(chain):
        _, cl, P, cr = blk.shape
        if j == len(chain) - 1:
            out.append(blk.reshape(nb * cl, P, cr))
        else:
            T = torch.zeros((nb, cl, P, nb, cr), dtype=blk.dtype, device=blk.device)
            T[ar, :, :, ar, :] = blk
            out.append(T.reshape(nb * cl, P, nb * cr))
    return out


class GaussianPTBuilderGPU:
    """ptgen.GaussianPTBuilder with the tail in device memory and the compressions on the GPU (module docstring).
    The constants (coupling structure, trace-adapted basis, bath factors) are the host builder's, moved to the
    device once."""

    def __init__(self, boson_op, eta, delta_pol=0.0, dt=None, threshold=1e-10, max_bond=64,
                 subtract_polaron_shift=True, tail_threshold=None, tail_max_bond=None, trace_basis=True,
                 tail="qrcp", device=None):
        torch = _torch()
        self.torch = torch
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        h = ptgen.GaussianPTBuilder(boson_op, eta, delta_pol, dt, threshold, max_bond, subtract_polaron_shift,
                                    tail_threshold, tail_max_bond, trace_basis)
        self.host = h
        self.gmap, self.pairs, self.xis = h.gmap, h.pairs, h.xis
        self.K, self.D, self.P, self.nl = h.K, h.D, h.P, h.nl
        self.threshold, self.tail_threshold = h.threshold, h.tail_threshold
        self.max_bond, self.tail_max_bond = max_bond, tail_max_bond
        self.tail_mode = tail
        self.pair_ip, self.pair_im = h.pair_ip, h.pair_im
        d = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.complex128, device=self.dev)  # noqa: E731
        self.cvec = d(h.cvec)
        self.reindex = d(h.reindex)
        self.phi = d(h.phi)
        self.Fp, self.Fm = d(h.Fp), d(h.Fm)
        self.newp = d(h.newp) if h.newp is not None else None
        self.tail = [d(t) for t in h.tail]
        self.r = 1
        self.trunc = ptgen.TruncationStats(self.threshold, max_bond)
        self._ip = torch.as_tensor(self.pair_ip, device=self.dev)
        self._im = torch.as_tensor(self.pair_im, device=self.dev)

    def closure(self, tail=None):
        torch = self.torch
        tail = self.tail if tail is None else tail
        if not tail:
            return np.ones(1, dtype=np.complex128)
        v = torch.einsum("p,lpr->lr", self.cvec, tail[-1])
        for T in reversed(tail[:-1]):
            v = torch.einsum("p,lpr->lr", self.cvec, T) @ v
        return v[:, 0].cpu().numpy()

    def _advance(self, tail):
        torch = self.torch
        nl, K = self.nl, self.K
        r = tail[0].shape[0]
        first = torch.einsum("ims,bsc->ibmc", self.reindex, tail[0])
        st = _stack(first, tail[1:], self.Fp[:, : K - 1], self.newp)
        Up, chain = _compress(st, self.threshold, self.max_bond, self.tail_threshold, self.tail_max_bond,
                              self.tail_mode, self.trunc)
        r1 = Up.shape[1]
        pres = chain[0]
        nxt = torch.einsum("bpq,lqr->blpr", self.Fm[:, 0], chain[1])
        first = torch.einsum("ibc,icpr->ibpr", pres.permute(1, 0, 2), nxt)
        st = _stack(first, chain[2:], self.Fm[:, 1:K], None)
        Um, tail2 = _compress(st, self.threshold, self.max_bond, self.tail_threshold, self.tail_max_bond,
                              self.tail_mode, self.trunc)
        return Up.reshape(nl, r, r1), Um.reshape(nl, r1, Um.shape[1]), tail2

    def _slice(self, Up, Um):
        return self.phi[:, None, None] * (Up[self._ip] @ Um[self._im])

    def step(self):
        """one PT slice: (Q[D, r, r'] numpy, closure[r'] numpy)"""
        if self.K == 0:
            return np.asarray(self.host.phi)[:, None, None].astype(np.complex128), np.ones(1, dtype=np.complex128)
        Up, Um, tail = self._advance(self.tail)
        self.tail, self.r = tail, tail[0].shape[0]
        return self._slice(Up, Um).cpu().numpy(), self.closure()

    def stationary_slice(self):
        """ptgen.GaussianPTBuilder.stationary_slice on the device (the least-squares projection through the same
        QR + Jacobi SVD, singular values below 1e-13 * max dropped as numpy.linalg.lstsq(rcond=1e-13) does)."""
        torch = self.torch
        if self.K == 0:
            return np.asarray(self.host.phi)[:, None, None].astype(np.complex128)
        W0 = [t.clone() for t in self.tail]
        Up, Um, W1 = self._advance([t.clone() for t in self.tail])
        Q = self._slice(Up, Um)
        W = [t.clone() for t in W0]
        _rcanon(W)
        e = torch.ones((1, 1), dtype=torch.complex128, device=self.dev)
        for Tw, Tx in zip(reversed(W[1:]), reversed(W1[1:])):
            e = torch.einsum("apx,xy,bpy->ab", Tw.conj(), e, Tx)
        Op = torch.einsum("rpy,cy->rpc", W1[0], e).reshape(W1[0].shape[0], -1)
        L = W[0].reshape(W[0].shape[0], -1)
        U, S, Vh = svd(L.T)                      # L^T X = Op^T  (least squares)
        keep = S > 1e-13 * S[0]
        Sinv = torch.where(keep, 1.0 / torch.where(keep, S, torch.ones_like(S)), torch.zeros_like(S))
        X = Vh.conj().T @ (Sinv[:, None].to(U.dtype) * (U.conj().T @ Op.T))
        R = X.T
        self.stationary_residual = float(torch.linalg.norm(R @ L - Op) / max(float(torch.linalg.norm(Op)), 1e-300))
        return torch.einsum("gab,bc->gac", Q, R).cpu().numpy()


def build_gaussian_pt_gpu(boson_op, dt, eta, delta_pol=0.0, n_init=None, threshold=1e-10, max_bond=64, repeat=True,
                          subtract_polaron_shift=True, verbose=False, tail_max_bond=None, tail="qrcp", **builder_kw):
    """ptgen.build_gaussian_pt with the GPU builder: n_init explicit slices (default 2 K, ACE's `te 2*t_mem`) and,
    with repeat=True, one stationary slice repeated forever. Returns a host ProcessTensor."""
    b = GaussianPTBuilderGPU(boson_op, eta, delta_pol, dt, threshold, max_bond, subtract_polaron_shift,
                             tail_max_bond=tail_max_bond, tail=tail, **builder_kw)
    K = b.K
    n_init = 2 * max(K, 1) if n_init is None else int(n_init)
    Qs, cls = [], []
    for n in range(n_init):
        Q, c = b.step()
        Qs.append(Q)
        cls.append(c)
        if verbose and (n % 50 == 0 or n == n_init - 1):
            print(f"ptgen_gpu: step {n + 1}/{n_init} bond {b.r}", flush=True)
    if repeat:
        cls.append(b.closure())
        Qs.append(b.stationary_slice())
    chi = max(max(q.shape[1], q.shape[2]) for q in Qs)
    S = len(Qs)
    Qp = np.zeros((S, b.D, chi, chi), dtype=np.complex128)
    Cp = np.zeros((S, chi), dtype=np.complex128)
    for s, (q, c) in enumerate(zip(Qs, cls)):
        Qp[s, :, : q.shape[1], : q.shape[2]] = q
        Cp[s, : c.shape[0]] = c
    e0 = np.zeros(chi, dtype=np.complex128)
    e0[0] = 1.0
    b.trunc.warn("ptgen_gpu")
    return ProcessTensor(Q=Qp, closure=Cp, closure0=e0, bond0=e0, gmap=b.gmap,
                         n_init=n_init if repeat else S - 1, dt=dt, meta={"truncation": b.trunc.as_meta()})


def qd_phonon_pt_gpu(boson_op, dt, t_mem=20.48, ae=3.0, temperature=1.0, threshold=1e-10, factor_ah=None,
                     boson_e_max=7.0, J_file=None, use_infinite=False, max_bond=None, n_init=None, verbose=False,
                     tail="qrcp", K=None):
    """ptgen.qd_phonon_pt on the GPU: the PT of general_system.py:152-211's generate file, from its parameters (memory
    t_mem, or the bath's own memory with use_infinite: ptgen.infinite_memory_steps). Carries `meta`."""
    if max_bond is None:
        max_bond = ptgen.default_max_bond(boson_op)
    eta, delta, info = ptgen.qd_phonon_eta(boson_op, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max,
                                           J_file, use_infinite, K)
    if verbose and use_infinite:
        print("ptgen_gpu: infinite memory K = {} steps ({})".format(
            info["K"], "converged" if info.get("converged", True) else "capped at te = 2 t_mem"), flush=True)
    pt = build_gaussian_pt_gpu(boson_op, dt, eta, delta, n_init=n_init, threshold=threshold, max_bond=max_bond,
                               repeat=True, verbose=verbose, tail=tail)
    pt.meta = dict(ptgen.generation_key(boson_op, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max,
                                        J_file, use_infinite, max_bond), generator="gpu", tail=tail, **info,
                   truncation=(pt.meta or {}).get("truncation"))
    return pt
