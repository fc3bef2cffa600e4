"""Gaussian-bath process-tensor generator: the PT that `ACE <generate.param>` writes with `write_PT`.

Replaces the reference's PT-generation shell-out (pyaceqd/general_system/general_system.py:152-211: `dt`, `te
2*t_mem`, `threshold 1e-<threshold>`, `t_mem`, `use_Gaussian_repeat` / `use_Gaussian_infinite`,
`Boson_subtract_polaron_shift true`, `Boson_E_min 0`, `Boson_E_max <boson_e_max>`, `Boson_SysOp {boson_op}`,
`Boson_J_type QDPhonon`, `Boson_J_a_e <ae>`, `Boson_J_a_h <ae/factor_ah>`, `Boson_J_from_file`, `Boson_J_print`,
`temperature`). ACE itself is external and absent, so the PT it would write is unpinned; this
module is pinned instead by (tests/test_ptgen.py):
  * the exact independent-boson (pure dephasing) solution, which the discretised influence functional reproduces
    at any dt when the memory covers the whole run;
  * an exact, uncompressed shift-register PT (oracle/ptgen_oracle.py) for short memories with driving.

Physics (all frequencies in 1/ps, energies in meV, hbar = 0.6582119569 meV ps):
  H_I = A (x) sum_q g_q (b_q + b_q^dag), A = Boson_SysOp (diagonal, eigenvalues lambda_i; every pyaceqd model's
  boson_op is diagonal: tls.py:56, four_level_system/linear.py:17, six_level_system/linear.py:50).
  J(omega) = sum_q g_q^2 delta(omega - omega_q); C(t) = int J(w) [coth(hbar w / 2kT) cos wt - i sin wt] dw.
  Liouville index alpha = (i, j) has ket/bra eigenvalues (s+, s-) = (lambda_i, lambda_j), xi = s+ - s-.
  Step n (the PT slice sits between the two symmetric-Trotter half steps) contributes
      prod_{k=0..K} exp(-xi_n (eta_k s+_{n-k} - conj(eta_k) s-_{n-k}))
  with eta_0 = int_0^dt dt' int_0^t' dt'' C(t'-t''), eta_k = int_0^dt int_0^dt C(k dt + t' - t'') (Makri's QUAPI
  coefficients, computed by quadrature of J on [E_min, E_max]/hbar), K = round(t_mem / dt). Subtracting the
  polaron shift Delta = int J(w)/w dw adds +hbar Delta A^2 to H_S: a factor exp(-i Delta dt (s+^2 - s-^2)).

PT-MPO construction ("future-influence" form). After step n the bond carries the influence of the past on the
next K steps, a function v(xi_{n+1}, ..., xi_{n+K}); it is held as an MPS over those K future sites (physical
dimension P = number of distinct xi values) whose left boundary index is the PT bond b. Step n+1 with pair alpha:
  * site 1 (the present) is projected onto xi(alpha);
  * every remaining future site k = 1..K-1 is multiplied by exp(-xi (eta_k s+ - conj(eta_k) s-));
  * a new site k = K is appended (a product factor);
  * the stacked object over (b, alpha) is compressed by SVD: right-canonical QR sweep, boundary SVD (its left
    factor, an isometry over (b, alpha), is the PT slice Q[alpha] = phi(alpha) U[(b, alpha), b']), then a
    truncating left-to-right SVD sweep over the tail. Singular values below threshold * sigma_max are dropped.
The closure after a step is the tail evaluated on the trace (xi = 0 on every future site). The slice is stationary
once n >= K; `use_Gaussian_repeat` keeps n_init = 2K explicit slices and one repeated slice, projected onto the
fixed bond basis of the stationary tail (so the repeated slice maps that basis onto itself).
"""
import os

import numpy as np

from .constants import hbar as HBAR
from .engine import ProcessTensor

KB = 0.08617333262  # Boltzmann constant, meV/K

# QDPhonon: LA-phonon deformation-potential coupling of a GaAs quantum dot with Gaussian electron/hole
# wave functions (Krummheuer/Axt/Kuhn form). ACE's own defaults are not visible from the reference; these are the
# standard GaAs values and are stated here so they can be checked.
QD_RHO = 5370.0          # kg/m^3
QD_CS = 5110.0           # m/s
QD_DE = 7.0              # eV
QD_DH = -3.5             # eV
QD_AH_FACTOR = 1.15      # a_h = a_e / 1.15 when Boson_J_a_h is not given
_EV = 1.602176634e-19
_HBAR_SI = 1.054571817e-34


def qd_phonon_J(omega, ae=3.0, ah=None, D_e=QD_DE, D_h=QD_DH, rho=QD_RHO, c_s=QD_CS):
    """J(omega) in 1/ps for omega in 1/ps (ae, ah in nm):
    J = omega^3 (D_e exp(-w^2 a_e^2 / 4c^2) - D_h exp(-w^2 a_h^2 / 4c^2))^2 / (4 pi^2 rho hbar c^5)."""
    ah = ae / QD_AH_FACTOR if ah is None else ah
    w = np.asarray(omega, dtype=np.float64) * 1e12
    ff = (D_e * np.exp(-(w * ae * 1e-9) ** 2 / (4 * c_s ** 2)) - D_h * np.exp(-(w * ah * 1e-9) ** 2 / (4 * c_s ** 2)))
    return w ** 3 * (ff * _EV) ** 2 / (4 * np.pi ** 2 * rho * _HBAR_SI * c_s ** 5) * 1e-12


def write_J(path, J, e_min=0.0, e_max=15.0, n=2000):
    """`Boson_J_print <file> 0 15 2000` (general_system.py:186-187): columns omega [1/ps], J(omega) [1/ps]."""
    w = np.linspace(e_min, e_max, n) / HBAR
    np.savetxt(path, np.column_stack([w, J(w)]))


def J_from_file(path):
    """`Boson_J_from_file` (general_system.py:178-179): two columns omega [1/ps], J [1/ps]; linear interpolation,
    zero outside the tabulated range."""
    d = np.loadtxt(path)
    w, j = d[:, 0], d[:, 1]
    return lambda om: np.interp(om, w, j, left=0.0, right=0.0)


def eta_coefficients(J, temperature, dt, n_mem, e_min=0.0, e_max=7.0, n_omega=1 << 16):
    """(eta[0..n_mem], polaron shift Delta [1/ps]) by Simpson quadrature of J on [e_min, e_max]/hbar."""
    n = n_omega + 1 if n_omega % 2 == 0 else n_omega
    w = np.linspace(e_min / HBAR, e_max / HBAR, n)
    h = w[1] - w[0]
    sw = np.ones(n)
    sw[1:-1:2], sw[2:-1:2] = 4.0, 2.0
    sw *= h / 3
    Jw = np.asarray(J(w), dtype=np.float64)
    nz = w > 0
    if temperature > 0:
        x = HBAR * w[nz] / (2 * KB * temperature)
        coth = np.ones_like(w)
        coth[nz] = 1.0 / np.tanh(x)
    else:
        coth = np.ones_like(w)
    inv2 = np.zeros_like(w)
    inv2[nz] = 1.0 / w[nz] ** 2
    a = Jw * inv2 * sw   # J / w^2 dw
    eta = np.zeros(n_mem + 1, dtype=np.complex128)
    wd = w * dt
    eta[0] = np.sum(a * (coth * (1 - np.cos(wd)) + 1j * (np.sin(wd) - wd)))
    s2 = 4 * np.sin(wd / 2) ** 2
    for k in range(1, n_mem + 1):
        eta[k] = np.sum(a * s2 * (coth * np.cos(k * wd) - 1j * np.sin(k * wd)))
    inv1 = np.zeros_like(w)
    inv1[nz] = 1.0 / w[nz]
    delta = float(np.sum(Jw * inv1 * sw))
    return eta, delta


def _coupling_structure(boson_op, decimals=12):
    B = np.asarray(boson_op)
    if not np.allclose(B, np.diag(np.diag(B))):
        raise ValueError("only diagonal system-bath couplings are supported (all pyaceqd models are)")
    lam = np.round(np.real(np.diag(B)), decimals)
    N = len(lam)
    pairs, gmap = [], np.zeros(N * N, dtype=np.int32)
    for i in range(N):
        for j in range(N):
            key = (lam[i], lam[j])
            if key not in pairs:
                pairs.append(key)
            gmap[i * N + j] = pairs.index(key)
    xis = sorted({round(a - b, decimals) for a, b in pairs})
    return gmap, pairs, np.array(xis, dtype=np.float64)


def _rcanon(mps):
    """right-canonical QR sweep over sites len-1 .. 1 (site 0 keeps the norm)"""
    for j in range(len(mps) - 1, 0, -1):
        T = mps[j]
        cl, P, cr = T.shape
        q, r = np.linalg.qr(T.reshape(cl, P * cr).conj().T)
        k = q.shape[1]
        mps[j] = q.conj().T.reshape(k, P, cr)
        mps[j - 1] = np.tensordot(mps[j - 1], r.conj().T, axes=(2, 0))


def _keep(S, threshold, max_k):
    if S.size == 0 or S[0] == 0:
        return 1
    k = int(np.count_nonzero(S > threshold * S[0]))
    return max(1, min(k, max_k) if max_k else k)


class TruncationStats:
    """What decided the boundary cuts of one generation: the caller's threshold keeps every
    singular value above threshold x sigma_1 (ACE's `threshold`, general_system.py:159-190), the bond cap (the sweep
    kernel's LDS bond, default_max_bond) may cut below that. Recorded per boundary SVD: how many cuts the cap made
    (cap_bound), the largest rank the threshold asked for, and the largest discarded singular value relative to
    sigma_1 (max_discarded_rel: at most the threshold where the threshold decided every cut)."""

    def __init__(self, threshold, max_bond):
        self.threshold, self.max_bond = float(threshold), max_bond
        self.compressions = 0
        self.cap_bound = 0
        self.max_rank_wanted = 0
        self.max_discarded_rel = 0.0

    def record(self, S, k):
        S = np.asarray(S)
        if S.size == 0 or S[0] == 0:
            return
        self.compressions += 1
        want = int(np.count_nonzero(S > self.threshold * S[0]))
        self.max_rank_wanted = max(self.max_rank_wanted, want)
        if self.max_bond and want > self.max_bond:
            self.cap_bound += 1
        if k < S.size:
            self.max_discarded_rel = max(self.max_discarded_rel, float(S[k] / S[0]))

    def as_meta(self):
        return {"compressions": self.compressions, "cap_bound": self.cap_bound,
                "max_rank_wanted": self.max_rank_wanted, "max_discarded_rel": self.max_discarded_rel,
                "cap_decided": self.cap_bound > 0}

    def warn(self, where):
        """warnings.warn when the cap, not the threshold, set any cut"""
        if self.cap_bound:
            import warnings
            warnings.warn(f"{where}: the bond cap {self.max_bond} (the sweep kernel's bond) cut {self.cap_bound} of "
                          f"{self.compressions} boundary SVDs below the threshold {self.threshold:g}: the threshold "
                          f"asked for bonds up to {self.max_rank_wanted}; largest discarded singular value "
                          f"{self.max_discarded_rel:.2e} of sigma_1 (recorded in pt.meta['truncation'])",
                          RuntimeWarning, stacklevel=3)


def _fix_phase(U, Vh):
    """deterministic gauge: the largest-|.| entry of every left singular vector is real positive"""
    idx = np.argmax(np.abs(U), axis=0)
    ph = U[idx, np.arange(U.shape[1])]
    ph = ph / np.maximum(np.abs(ph), 1e-300)
    return U * ph.conj()[None, :], Vh * ph[:, None]


def _compress(mps, threshold, max_bond, tail_threshold=None, tail_max_bond=None, stats=None):
    """mps[0] has the (stacked) left boundary as its left index. Returns (U, mps') with U the isometry of the
    boundary SVD (left dim x new bond) and mps' the compressed tail whose left index is the new bond. `stats`
    (TruncationStats) records what decided the boundary cut."""
    tthr = threshold if tail_threshold is None else tail_threshold
    _rcanon(mps)
    T = mps[0]
    L, P, cr = T.shape
    U, S, Vh = np.linalg.svd(T.reshape(L, P * cr), full_matrices=False)
    k = _keep(S, threshold, max_bond)
    if stats is not None:
        stats.record(S, k)
    U, Vh = _fix_phase(U[:, :k], Vh[:k])
    cur = (S[:k, None] * Vh).reshape(k, P, cr)
    for j in range(len(mps) - 1):
        cl, P, cr = cur.shape
        u, s, vh = np.linalg.svd(cur.reshape(cl * P, cr), full_matrices=False)
        kk = _keep(s, tthr, tail_max_bond)
        mps[j] = u[:, :kk].reshape(cl, P, kk)
        cur = np.tensordot(s[:kk, None] * vh[:kk], mps[j + 1], axes=(1, 0))
    mps[-1] = cur
    return U, mps


def _stack(first, later, F, new):
    """Direct sum over blocks beta of the chains [first[beta], F[beta, j] later[j] ..., new[beta]] with the
    boundary rows (beta, b): block-diagonal bonds, the last site concatenated vertically.
    first: (nb, r, P1, c1); later: shared site tensors; F: (nb, len(later), P, P); new: (nb, P) or None."""
    nb, r, P1, c1 = first.shape
    chain = [first] + [np.einsum("bpq,lqr->blpr", F[:, j], T) for j, T in enumerate(later)]
    if new is not None:
        chain.append(new[:, None, :, None])
    out = []
    for j, blk in enumerate(chain):
        _, cl, P, cr = blk.shape
        if j == len(chain) - 1:
            out.append(blk.reshape(nb * cl, P, cr))
        else:
            T = np.zeros((nb, cl, P, nb, cr), dtype=np.complex128)
            for b in range(nb):
                T[b, :, :, b, :] = blk[b]
            out.append(T.reshape(nb * cl, P, nb * cr))
    return out


class GaussianPTBuilder:
    """Sequential PT-MPO builder (see module docstring). Holds the future-influence tail between steps.

    Future sites are stored in a trace-adapted basis: a site function f(xi) is kept as g = B f with g[0] = f(0)
    and g[xi] = f(xi) - f(0) (xi != 0). The trace closure is then e_0 with norm 1 while the bath factors
    exp(-xi z) ~ 1 + O(eta) are (1, O(eta), ...): the Frobenius norm that the SVD truncates in weighs the closure
    direction like every other, instead of sqrt(P) times less per future site (which made the truncation error
    of an observable ~ P^(K/2) x threshold in the plain xi basis).

    One step is split into an s+ half and an s- half (the bath factor exp(-xi (eta s+ - conj(eta) s-)) factorises):
    the s+ half stacks n_lambda blocks (one per distinct coupling eigenvalue of the ket), keeps the present site
    open with the bra eigenvalue as its index and compresses; the s- half projects the present site, stacks
    n_lambda blocks again and compresses. Q[(s+, s-)] = phi U+[s+] U-[s-]. Each compression stacks n_lambda
    instead of n_lambda^2 blocks: (n_lambda c)^3 instead of (n_lambda^2 c)^3 per site."""

    def __init__(self, boson_op, eta, delta_pol=0.0, dt=None, threshold=1e-10, max_bond=64,
                 subtract_polaron_shift=True, tail_threshold=None, tail_max_bond=None, trace_basis=True):
        self.gmap, self.pairs, self.xis = _coupling_structure(boson_op)
        self.eta = np.asarray(eta, dtype=np.complex128)
        self.K = len(self.eta) - 1
        self.dt = dt
        self.threshold = float(threshold)
        self.tail_threshold = self.threshold if tail_threshold is None else float(tail_threshold)
        self.max_bond = max_bond
        self.tail_max_bond = tail_max_bond
        self.D, P = len(self.pairs), len(self.xis)
        self.P = P
        lams = sorted({p[0] for p in self.pairs})
        self.lams = np.array(lams)
        nl = len(lams)
        self.nl = nl
        lam_idx = {v: i for i, v in enumerate(lams)}
        self.pair_ip = np.array([lam_idx[p[0]] for p in self.pairs])
        self.pair_im = np.array([lam_idx[p[1]] for p in self.pairs])
        x0 = int(np.argmin(np.abs(self.xis)))
        order = [x0] + [q for q in range(P) if q != x0]       # xi = 0 is basis element 0
        self.xis = self.xis[order]
        Bm = np.eye(P, dtype=np.complex128)
        Binv = np.eye(P, dtype=np.complex128)
        if trace_basis:
            Bm[1:, 0] = -1.0
            Binv[1:, 0] = 1.0
        self.B, self.Binv = Bm, Binv
        self.one = Bm @ np.ones(P, dtype=np.complex128)         # the constant function (no past) in this basis
        self.cvec = Binv[0]                                      # f(0) = cvec . g: the trace closure
        xi_of = np.array([[int(np.argmin(np.abs(self.xis - (a - b)))) for b in lams] for a in lams])  # [ip, im]
        self.reindex = Binv[xi_of]                               # (ip, im, P): f(lam_ip - lam_im) = . g
        sp = np.array([p[0] for p in self.pairs])
        sm = np.array([p[1] for p in self.pairs])
        xi_a = sp - sm
        ph = 0.0 if not subtract_polaron_shift or dt is None else delta_pol * dt
        self.phi = np.exp(-xi_a * (self.eta[0] * sp - np.conj(self.eta[0]) * sm) - 1j * ph * (sp ** 2 - sm ** 2))
        L = self.lams
        e = self.eta[1:]
        dplus = np.exp(-self.xis[None, None, :] * (e[None, :, None] * L[:, None, None]))             # (nl, K, P)
        dminus = np.exp(self.xis[None, None, :] * (np.conj(e)[None, :, None] * L[:, None, None]))
        self.Fp = np.einsum("pq,akq,qr->akpr", Bm, dplus, Binv, optimize=True)                   # (nl, K, P, P)
        self.Fm = np.einsum("pq,akq,qr->akpr", Bm, dminus, Binv, optimize=True)
        self.newp = np.einsum("pq,aq->ap", Bm, dplus[:, -1, :]) if self.K else None              # (nl, P)
        self.tail = [self.one.reshape(1, P, 1).copy() for _ in range(self.K)]
        self.r = 1
        self.trunc = TruncationStats(self.threshold, max_bond)

    def closure(self, tail=None):
        tail = self.tail if tail is None else tail
        if not tail:
            return np.ones(1, dtype=np.complex128)
        v = np.einsum("p,lpr->lr", self.cvec, tail[-1])
        for T in reversed(tail[:-1]):
            v = np.einsum("p,lpr->lr", self.cvec, T) @ v
        return v[:, 0]

    def _advance(self, tail):
        """(U+ (nl, r, r'), U- (nl, r', r''), new tail) for one step from `tail`"""
        nl, K = self.nl, self.K
        r = tail[0].shape[0]
        # s+ half: present site re-indexed by s-, futures k = 1..K-1 and the new site k = K times the s+ factor
        first = np.einsum("ims,bsc->ibmc", self.reindex, tail[0])              # (nl, r, nl, c1)
        st = _stack(first, tail[1:], self.Fp[:, : K - 1], self.newp)
        Up, chain = _compress(st, self.threshold, self.max_bond, self.tail_threshold, self.tail_max_bond, self.trunc)
        r1 = Up.shape[1]
        # s- half: project the present site onto s-, every future site (incl. the new one) times the s- factor
        pres = chain[0]                                                         # (r1, nl, c1)
        nxt = np.einsum("bpq,lqr->blpr", self.Fm[:, 0], chain[1])               # (nl, c1, P, c2)
        first = np.einsum("ibc,icpr->ibpr", pres.transpose(1, 0, 2), nxt)       # (nl, r1, P, c2)
        st = _stack(first, chain[2:], self.Fm[:, 1:K], None)
        Um, tail2 = _compress(st, self.threshold, self.max_bond, self.tail_threshold, self.tail_max_bond, self.trunc)
        return Up.reshape(nl, r, r1), Um.reshape(nl, r1, Um.shape[1]), tail2

    def _slice(self, Up, Um):
        return np.stack([self.phi[g] * (Up[self.pair_ip[g]] @ Um[self.pair_im[g]]) for g in range(self.D)])

    def step(self):
        """one PT slice: returns (Q[D, r, r'], closure[r'])"""
        if self.K == 0:
            return self.phi[:, None, None].astype(np.complex128), np.ones(1, dtype=np.complex128)
        Up, Um, tail = self._advance(self.tail)
        self.tail, self.r = tail, tail[0].shape[0]
        return self._slice(Up, Um), self.closure()

    def stationary_slice(self):
        """Q[alpha] of the stationary regime in the CURRENT bond basis (the tail W): one more step gives
        Q (W basis -> W' basis) and W'; W' is expressed in W (W'_b'' = sum_b R[b'', b] W_b, least squares with W
        in right-canonical form W = L R_basis, so the conditioning is that of L's singular values) and the slice
        Q R maps the W basis onto itself. Leaves the builder state unchanged."""
        if self.K == 0:
            return self.phi[:, None, None].astype(np.complex128)
        W0 = [t.copy() for t in self.tail]
        Up, Um, W1 = self._advance([t.copy() for t in self.tail])
        Q = self._slice(Up, Um)
        W = [t.copy() for t in W0]
        _rcanon(W)
        e = np.ones((1, 1), dtype=np.complex128)
        for Tw, Tx in zip(reversed(W[1:]), reversed(W1[1:])):
            e = np.einsum("apx,xy,bpy->ab", Tw.conj(), e, Tx, optimize=True)   # <Rtail_c | W1tail_c'>
        Op = np.einsum("rpy,cy->rpc", W1[0], e).reshape(W1[0].shape[0], -1)     # <R_(p,c) | W1_b''>
        L = W[0].reshape(W[0].shape[0], -1)
        R = np.linalg.lstsq(L.T, Op.T, rcond=1e-13)[0].T                      # (r'', r)
        self.stationary_residual = float(np.linalg.norm(R @ L - Op) / max(np.linalg.norm(Op), 1e-300))
        return np.einsum("gab,bc->gac", Q, R)


def build_gaussian_pt(boson_op, dt, eta, delta_pol=0.0, n_init=None, threshold=1e-10, max_bond=64, repeat=True,
                      subtract_polaron_shift=True, verbose=False, tail_max_bond=None, **builder_kw):
    """ProcessTensor with n_init explicit slices and (repeat=True) one stationary slice repeated forever.
    n_init defaults to 2 K (ACE: `te 2*t_mem`, general_system.py:160)."""
    b = GaussianPTBuilder(boson_op, eta, delta_pol, dt, threshold, max_bond, subtract_polaron_shift,
                          tail_max_bond=tail_max_bond, **builder_kw)
    K = b.K
    n_init = 2 * max(K, 1) if n_init is None else int(n_init)
    Qs, cls = [], []
    for n in range(n_init):
        Q, c = b.step()
        Qs.append(Q)
        cls.append(c)
        if verbose and (n % 50 == 0 or n == n_init - 1):
            print(f"ptgen: step {n + 1}/{n_init} bond {b.r}")
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
    b.trunc.warn("ptgen")
    return ProcessTensor(Q=Qp, closure=Cp, closure0=e0, bond0=e0, gmap=b.gmap,
                         n_init=n_init if repeat else S - 1, dt=dt, meta={"truncation": b.trunc.as_meta()})


def infinite_memory_steps(eta, boson_op, threshold):
    """Memory K (in steps) of the `use_Gaussian_infinite` PT (general_system.py:150-151, 165-167: no `t_mem` line, the
    generate file keeps `te 2*t_mem` and `threshold`). ACE's infinite-memory construction is not visible offline; here
    the memory is the bath's own: the shortest K whose neglected couplings cannot move an influence value by more than
    the compression threshold per step,
        max|xi| max|lambda| sum_{k = K+1 .. k_cap} |eta_k| <= threshold,
    with eta computed to k_cap = len(eta) - 1 = round(2 t_mem / dt), the `te` horizon the generate file still writes
    (ACE propagates the generation to te, so no correlation longer than te can enter its PT either). Returns
    (K, converged): converged is False when the tail never drops below the threshold inside te (K = k_cap then;
    e.g. a_e = 3 nm, whose eta_k keep a ~1e-9 floor from the hard Boson_E_max cut of J)."""
    lam = np.real(np.diag(np.asarray(boson_op)))
    s = float(np.max(np.abs(lam))) * float(np.max(np.abs(lam[:, None] - lam[None, :])))
    a = np.abs(np.asarray(eta)[1:])
    k_cap = len(a)
    if k_cap == 0 or s == 0.0:
        return max(k_cap, 0), True
    tail = np.concatenate([np.cumsum(a[::-1])[::-1], [0.0]])       # tail[K] = sum_{k > K} |eta_k|, K = 0..k_cap
    K = int(np.nonzero(s * tail <= threshold)[0][0])              # tail[k_cap] = 0: always found
    return max(1, K), K < k_cap


def qd_phonon_eta(boson_op, dt, t_mem=20.48, ae=3.0, temperature=1.0, threshold=1e-10, factor_ah=None,
                  boson_e_max=7.0, J_file=None, use_infinite=False, K=None):
    """(eta[0..K], polaron shift, info) of the generate file's bath: J from QDPhonon(a_e, a_h) or `Boson_J_from_file`,
    memory K = round(t_mem / dt) (`t_mem`, use_Gaussian_repeat) or infinite_memory_steps (use_Gaussian_infinite).
    K (int) overrides the memory (the memory-convergence tests)."""
    if J_file is not None:
        J = J_from_file(J_file)
    else:
        ah = None if factor_ah is None else ae / factor_ah
        J = lambda w: qd_phonon_J(w, ae=ae, ah=ah)  # noqa: E731
    info = {"infinite": bool(use_infinite)}
    if K is not None:
        n_mem = int(K)
    elif use_infinite:
        k_cap = max(1, int(round(2 * t_mem / dt)))
        eta, _ = eta_coefficients(J, temperature, dt, k_cap, e_max=boson_e_max)
        n_mem, conv = infinite_memory_steps(eta, boson_op, threshold)
        info.update(k_cap=k_cap, converged=bool(conv))
        if not conv:  # say it, not only in meta (a stand-in for ACE's use_Gaussian_infinite, parity unpinned)
            import warnings
            warnings.warn(f"use_infinite: the bath's eta_k tail stays above the threshold {threshold:g} up to the te "
                          f"horizon, so the memory is truncated at K = {n_mem} steps (2 t_mem / dt); this is a "
                          f"truncated-memory stand-in for ACE's use_Gaussian_infinite (parity unpinned)",
                          RuntimeWarning, stacklevel=2)
    else:
        n_mem = max(1, int(round(t_mem / dt)))
    eta, delta = eta_coefficients(J, temperature, dt, n_mem, e_max=boson_e_max)
    info["K"] = int(n_mem)
    return eta, delta, info


def generation_key(boson_op, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max, J_file, use_infinite,
                   max_bond):
    """The parameters that decide a generated PT (stored in its .npz as `meta`, compared when a cache is reused):
    coupling eigenvalues, dt, bath (a_e, a_h factor or the J file's content hash), temperature, threshold, E_max,
    memory mode (t_mem, or infinite: then t_mem only bounds the horizon te = 2 t_mem) and the bond cap."""
    import hashlib
    lam = [float(x) for x in np.round(np.real(np.diag(np.asarray(boson_op))), 12)]
    key = {"lam": lam, "dt": float(dt), "temperature": float(temperature), "threshold": float(threshold),
           "boson_e_max": float(boson_e_max), "infinite": bool(use_infinite), "t_mem": float(t_mem),
           "max_bond": int(max_bond)}
    if J_file is not None:
        with open(J_file, "rb") as f:
            key["J_sha1"] = hashlib.sha1(f.read()).hexdigest()
    else:
        key["ae"] = float(ae)
        key["factor_ah"] = None if factor_ah is None else float(factor_ah)
    return key


def default_max_bond(boson_op):
    """the bond cap of generated PTs: 128 for N <= 4, 64 above — the batched sweep kernel's LDS-resident bond
    (DESIGN.md §4). PQD_PT_MAX_BOND overrides it (0: no cap): bonds up to 256 at N <= 4 run on multi-trajectory
    split groups with the slice rows streamed (pt_msplit.hip, at most 8 trajectories per group), so a caller's
    threshold can decide the cut where the cap would (the cut is recorded in meta['truncation'])"""
    import os
    env = os.environ.get("PQD_PT_MAX_BOND")
    if env is not None and env.strip() != "":
        return int(env)
    return 128 if np.asarray(boson_op).shape[0] <= 4 else 64


def qd_phonon_pt(boson_op, dt, t_mem=20.48, ae=3.0, temperature=1.0, threshold=1e-10, factor_ah=None,
                 boson_e_max=7.0, J_file=None, use_infinite=False, max_bond=None, n_init=None, verbose=False, K=None):
    """The PT of general_system.py:152-211's generate file, from its own parameters: memory t_mem (repeat) or the
    bath's own memory (use_infinite, infinite_memory_steps). The bond is capped at what the sweep kernel holds in
    LDS: 128 for N <= 4, 64 above. The result carries its generation parameters in `meta`."""
    if max_bond is None:
        max_bond = default_max_bond(boson_op)
    eta, delta, info = qd_phonon_eta(boson_op, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max, J_file,
                                     use_infinite, K)
    if verbose and use_infinite:
        print("ptgen: infinite memory K = {} steps ({})".format(
            info["K"], "converged" if info.get("converged", True) else "capped at te = 2 t_mem"))
    pt = build_gaussian_pt(boson_op, dt, eta, delta, n_init=n_init, threshold=threshold, max_bond=max_bond,
                           repeat=True, verbose=verbose)
    pt.meta = dict(generation_key(boson_op, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max, J_file,
                                  use_infinite, max_bond), generator="host", tail="svd", **info,
                   truncation=(pt.meta or {}).get("truncation"))
    return pt


def pt_cache_name(system_prefix, ae, temperature, threshold, t_mem, dt, J_file=None, use_infinite=False):
    """general_system.py:146-151 naming (the pqd .npz container gets the suffix `.npz`)."""
    if use_infinite:
        name = "{}_{}k_th{}_dt{}.pt".format(system_prefix, temperature, threshold, dt)
    elif J_file is not None:
        name = "{}_{}_{}k_th{}_tmem{}_dt{}.ptr".format(system_prefix, os.path.splitext(J_file)[0], temperature,
                                                       threshold, t_mem, dt)
    else:
        name = "{}_{}nm_{}k_th{}_tmem{}_dt{}.ptr".format(system_prefix, ae, temperature, threshold, t_mem, dt)
    return name
