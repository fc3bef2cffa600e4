"""Exact (uncompressed) influence-functional PT — TEST INFRASTRUCTURE ONLY.

Checker for pyaceqd_amd/ptgen.py (the Gaussian-bath PT generator that replaces ACE's `write_PT`,
pyaceqd/general_system/general_system.py:152-211). ACE is absent, so the generator is pinned by
  * this shift-register PT: the discretised influence functional with memory K held exactly, the bond being the
    last K coupling-eigenvalue pairs (dimension (D+1)^K, the extra symbol marking "before t_start"), and
  * the closed-form independent-boson coherence (`ibm_coherence`), which the discretised influence functional
    reproduces at any dt.
Both restate the same physics as the generator's docstring (Makri's QUAPI eta_k with the slice between the two
symmetric-Trotter half steps; polaron-shift subtraction as exp(-i Delta dt (s+^2 - s-^2))), independently of its
MPS compression.
"""
import itertools

import numpy as np

from pyaceqd_amd.engine import ProcessTensor


def _pairs(boson_op, decimals=12):
    lam = np.round(np.real(np.diag(np.asarray(boson_op))), decimals)
    N = len(lam)
    pairs, gmap = [], np.zeros(N * N, dtype=np.int32)
    for i in range(N):
        for j in range(N):
            key = (lam[i], lam[j])
            if key not in pairs:
                pairs.append(key)
            gmap[i * N + j] = pairs.index(key)
    return gmap, pairs


def exact_if_pt(boson_op, eta, delta_pol=0.0, dt=None, subtract_polaron_shift=True):
    """Stationary shift-register PT: Q[a][(h_1..h_K), (a, h_1..h_{K-1})] = phi(a) prod_k b_k(a, h_k),
    b_k(a, h) = exp(-xi_a (eta_k s+_h - conj(eta_k) s-_h)); closure = all ones (the traced future contributes 1)."""
    gmap, pairs = _pairs(boson_op)
    D = len(pairs)
    eta = np.asarray(eta, dtype=np.complex128)
    K = len(eta) - 1
    sp = np.array([p[0] for p in pairs] + [0.0])     # symbol D = "no step yet": s+ = s- = 0
    sm = np.array([p[1] for p in pairs] + [0.0])
    xi = sp - sm
    ph = delta_pol * dt if (subtract_polaron_shift and dt is not None) else 0.0
    phi = np.exp(-xi[:D] * (eta[0] * sp[:D] - np.conj(eta[0]) * sm[:D]) - 1j * ph * (sp[:D] ** 2 - sm[:D] ** 2))
    S = D + 1
    chi = S ** K
    states = list(itertools.product(range(S), repeat=K))   # (h_1, ..., h_K), h_1 most recent
    index = {s: i for i, s in enumerate(states)}
    Q = np.zeros((1, D, chi, chi), dtype=np.complex128)
    for a in range(D):
        for i, h in enumerate(states):
            w = phi[a]
            for k in range(1, K + 1):
                hk = h[k - 1]
                w *= np.exp(-xi[a] * (eta[k] * sp[hk] - np.conj(eta[k]) * sm[hk]))
            j = index[(a,) + h[:-1]] if K else 0
            Q[0, a, i, j] = w
    bond0 = np.zeros(chi, dtype=np.complex128)
    bond0[index[(D,) * K] if K else 0] = 1.0
    ones = np.ones(chi, dtype=np.complex128)
    return ProcessTensor(Q=Q, closure=ones[None, :], closure0=ones, bond0=bond0, gmap=gmap, n_init=0, dt=dt)


def ibm_coherence_discrete(eta, delta_pol, dt, n_steps, rho10=0.5):
    """rho_10(t_n) of the independent-boson model (H_S = 0, A = |1><1|) from the discretised influence functional
    with memory K = len(eta)-1: exponent -sum_{j<n} sum_{k<=min(j,K)} eta_k, polaron shift subtracted."""
    K = len(eta) - 1
    csum = np.cumsum(eta)
    out = np.empty(n_steps + 1, dtype=np.complex128)
    E = 0.0
    out[0] = rho10
    for m in range(1, n_steps + 1):
        E = E + csum[min(m - 1, K)]
        out[m] = rho10 * np.exp(-E - 1j * delta_pol * dt * m)
    return out


def ibm_coherence_exact(J, temperature, times, e_max=7.0, n_omega=400001, rho10=0.5):
    """closed form: rho_10(t) = rho_10(0) exp(-int J/w^2 [coth(hbar w/2kT)(1 - cos wt) + i sin wt] dw)
    (polaron shift subtracted), trapezoid quadrature on an independent grid."""
    from pyaceqd_amd.constants import hbar
    kb = 0.08617333262
    w = np.linspace(0, e_max / hbar, n_omega)[1:]
    Jw = J(w)
    coth = 1.0 / np.tanh(hbar * w / (2 * kb * temperature)) if temperature > 0 else np.ones_like(w)
    res = []
    for t in np.atleast_1d(times):
        f = Jw / w ** 2 * (coth * (1 - np.cos(w * t)) + 1j * np.sin(w * t))
        res.append(rho10 * np.exp(-np.trapezoid(f, w)))
    return np.array(res)
