"""Process-tensor (PT-MPO) containers: on-disk format, dictionary map and synthetic generators.

The reference obtains its PTs from the external ACE binary (`dont_propagate true` + `write_PT`,
general_system.py:152-211) and points the propagation at them with `add_PT` (:236). That binary is
absent, so round 1 ships:
  * a documented .npz PT format (save_pt / load_pt) consumed by system_ace_stream(pt_file=...);
  * `pair_dictionary`: the diagonal-coupling dictionary g(alpha) from the boson operator's
    eigenvalues (every pyaceqd boson_op is diagonal: tls.py:56, four_level_system/linear.py:17,
    six_level_system/linear.py:50): Liouville indices alpha = (i, j) with equal eigenvalue pairs
    (lambda_i, lambda_j) share one chi x chi matrix;
  * `synthetic_pt`: the benchmark PT of SURVEY.md §8d (C2/C3/C4);
  * `markov_dephasing_pt`: an exactly solvable PT (pure dephasing encoded in the PT) used as a
    known-answer test against the equivalent Lindblad dissipator.
The Gaussian-bath PT generator itself (QDPhonon J(omega), SVD compression) is SURVEY.md §8f rank 1.
"""
import json

import numpy as np

from .engine import ProcessTensor


def pair_dictionary(boson_op, decimals=12, full=False):
    """gmap[alpha = i*N + j] -> index of the distinct eigenvalue pair (lambda_i, lambda_j).
    full=True gives every alpha its own entry (D = N^2, no dictionary compression)."""
    B = np.asarray(boson_op)
    if not np.allclose(B, np.diag(np.diag(B))):
        raise ValueError("only diagonal system-bath couplings are supported (all pyaceqd models are)")
    lam = np.round(np.real(np.diag(B)), decimals)
    N = len(lam)
    if full:
        return np.arange(N * N, dtype=np.int32), [(lam[a // N], lam[a % N]) for a in range(N * N)]
    pairs, gmap = [], np.zeros(N * N, dtype=np.int32)
    for i in range(N):
        for j in range(N):
            key = (lam[i], lam[j])
            if key not in pairs:
                pairs.append(key)
            gmap[i * N + j] = pairs.index(key)
    return gmap, pairs


def schedule_info(n_init, n_slices):
    return {"n_init": int(n_init), "n_slices": int(n_slices)}


def save_pt(path, pt: ProcessTensor, dim=None):
    """pqd-pt-v1 container. `meta` (the generation parameters, ptgen.generation_key) is stored as JSON text so a cached
    PT can be checked against the parameters of a later call (general_system._resolve_pt)."""
    meta = "" if pt.meta is None else json.dumps(pt.meta, sort_keys=True)
    np.savez(path, format="pqd-pt-v1", Q=pt.Q, closure=pt.closure, closure0=pt.closure0, bond0=pt.bond0,
             gmap=pt.gmap, n_init=pt.n_init, dt=np.nan if pt.dt is None else pt.dt,
             dim=-1 if dim is None else dim, meta=meta)


def load_pt(path) -> ProcessTensor:
    z = np.load(path, allow_pickle=False)
    if str(z["format"]) != "pqd-pt-v1":
        raise ValueError(f"{path}: not a pqd-pt-v1 file")
    dt = float(z["dt"])
    meta = str(z["meta"]) if "meta" in z.files else ""
    return ProcessTensor(Q=z["Q"], closure=z["closure"], closure0=z["closure0"], bond0=z["bond0"], gmap=z["gmap"],
                         n_init=int(z["n_init"]), dt=None if np.isnan(dt) else dt,
                         meta=json.loads(meta) if meta else None)


def synthetic_pt(boson_op, chi, n_init=1, n_rep=1, seed=1234, eps=0.05, structured=True, dictionary=False,
                 dt=None):
    """SURVEY.md §8d synthetic PT: per slice and dictionary entry M_g = I + eps G / sqrt(chi), G iid complex
    normal, rescaled to spectral radius <= 1. structured=True decouples bond channel 0 (Q[0,0] = 1, row/col 0
    otherwise 0) and uses closure = bond0 = e_0, so the physical outputs equal the bare (no-PT) dynamics
    exactly while the full chi x chi arithmetic is still performed (an end-to-end invariant)."""
    rng = np.random.default_rng(seed)
    gmap, pairs = pair_dictionary(boson_op, full=not dictionary)
    D = len(pairs)
    S = n_init + n_rep
    Q = np.empty((S, D, chi, chi), dtype=np.complex128)
    for s in range(S):
        for g in range(D):
            G = (rng.normal(size=(chi, chi)) + 1j * rng.normal(size=(chi, chi))) / np.sqrt(2.0)
            M = np.eye(chi) + eps * G / np.sqrt(chi)
            if structured:
                M[0, :] = 0
                M[:, 0] = 0
                M[0, 0] = 1
            rho = np.max(np.abs(np.linalg.eigvals(M)))
            Q[s, g] = M / max(1.0, rho)
            if structured:
                Q[s, g, 0, 0] = 1.0
    e0 = np.zeros(chi, dtype=np.complex128)
    e0[0] = 1
    closure = np.tile(e0, (S, 1))
    return ProcessTensor(Q=Q, closure=closure, closure0=e0, bond0=e0, gmap=gmap, n_init=n_init, dt=dt)


def random_pt(N, chi, D=None, n_slices=3, seed=0, eps=0.3):
    """Unstructured random PT (random closures and bond vector) for parity tests over short runs."""
    rng = np.random.default_rng(seed)
    D = D or N * N
    Q = np.eye(chi)[None, None] + eps * (rng.normal(size=(n_slices, D, chi, chi))
                                         + 1j * rng.normal(size=(n_slices, D, chi, chi))) / np.sqrt(2 * chi)
    cl = rng.normal(size=(n_slices, chi)) + 1j * rng.normal(size=(n_slices, chi))
    c0 = rng.normal(size=chi) + 1j * rng.normal(size=chi)
    b0 = rng.normal(size=chi) + 1j * rng.normal(size=chi)
    gmap = rng.integers(0, D, size=N * N).astype(np.int32)
    return ProcessTensor(Q=Q, closure=cl, closure0=c0, bond0=b0, gmap=gmap, n_init=n_slices - 1)


def markov_dephasing_pt(coupling_op, gamma, dt, chi=1):
    """Pure dephasing of rate gamma for the diagonal coupling operator A encoded as a (stationary, chi=1) PT:
    Q[g] = exp(-gamma/2 (lambda_i - lambda_j)^2 dt) — the exact one-step map of the Lindblad dissipator
    with L = A (rate gamma), which acts diagonally on |i><j|."""
    gmap, pairs = pair_dictionary(coupling_op)
    D = len(pairs)
    Q = np.zeros((1, D, chi, chi), dtype=np.complex128)
    for g, (li, lj) in enumerate(pairs):
        Q[0, g] = np.eye(chi) * np.exp(-0.5 * gamma * (li - lj) ** 2 * dt)
    one = np.zeros(chi, dtype=np.complex128)
    one[0] = 1
    return ProcessTensor(Q=Q, closure=one[None, :], closure0=one, bond0=one, gmap=gmap, n_init=0, dt=dt)
