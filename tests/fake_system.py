"""A deterministic stand-in for a pyaceqd model function (tls / biexciton / sixls_linear) — TEST INFRASTRUCTURE.

The caller modules (pol_entanglement.G2, two_time.*) only slice, integrate and combine what the model returns. To
pin that bookkeeping against the reference's own code, tests/golden/make_golden.py runs the reference classes with
`fake_system` in place of the ACE-backed model, and tests run ours with the same function. Every output row is an
analytic function of time, of the operator string and of the multi-time operators that have acted, so an index
slip or a swapped operator changes the numbers.

It accepts both call forms: the reference's one-trajectory call (returns [t, <op_1>, ..., <op_n>]) and the batched
`trajectories=[{"multitime_op", "t_end", "out_begin"}]` form of pyaceqd_amd.general_system (returns one
(1 + n_out, window) array per trajectory, window = steps out_begin..round(t_end/dt)).
"""
import numpy as np


def _h(s):
    return (sum((i + 1) * ord(c) for i, c in enumerate(str(s))) % 997) / 997.0


def fake_series(op, t, mtos):
    a = _h(op)
    v = (1 + a) * np.exp(-0.01 * (1 + a) * t) * np.exp(1j * (0.3 + a) * t)
    for m in mtos:
        tm = float(m["time"])
        b = _h(str(m["operator"]) + str(m.get("applyFrom", "")))
        on = (t >= tm - 1e-9).astype(float)
        v = v + on * (0.5 + b) * np.exp(-0.02 * (t - tm)) * np.exp(1j * b * (t - tm)) * (1 + 0.1 * tm)
    return v


def _run(t_start, t_end, dt, mtos, output_ops):
    n = int(round((t_end - t_start) / dt))
    t = t_start + dt * np.arange(n + 1)
    if isinstance(mtos, dict):
        mtos = [mtos]
    return np.array([t.astype(complex)] + [fake_series(o, t, mtos or []) for o in output_ops])


def fake_system(t_start, t_end, *pulses, dt=0.1, multitime_op=None, output_ops=[], trajectories=None, **kw):
    if trajectories is None:
        return _run(t_start, t_end, dt, multitime_op, output_ops)
    res = []
    for spec in trajectories:
        full = _run(t_start, spec.get("t_end", t_end), dt, spec.get("multitime_op"), output_ops)
        res.append(full[:, int(spec.get("out_begin", 0)):])
    return res


# ----------------------------------------------------------------------------- calc_dynmap=True
def _superop(A, kind, dim):
    """row-major vec: vec(A rho) = (A (x) I) vec(rho), vec(rho A) = (I (x) A^T) vec(rho)"""
    I = np.eye(dim)
    if kind == "_left":
        return np.kron(A, I)
    if kind == "_right":
        return np.kron(I, A.T)
    return np.kron(A, A.conj())


def fake_dynmaps(t_start, t_end, dt, mtos, dim, seed=5):
    """dm[k] = E(t_{k+1}, t_start) of a driven, damped dim-level system (random H0 + sin(0.7 t) H1, two jump
    operators); an MTO at step s (round((time - t_start)/dt)) acts before the step-s propagation"""
    import scipy.linalg as sla
    from pyaceqd_amd import opgrammar
    rng = np.random.default_rng(seed)
    H0 = rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))
    H0 = 0.5 * (H0 + H0.conj().T)
    H1 = rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))
    H1 = 0.5 * (H1 + H1.conj().T)
    Ls = [0.3 * (rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) for _ in range(2)]
    I = np.eye(dim)
    n = int(round((t_end - t_start) / dt))
    mt = [mtos] if isinstance(mtos, dict) else list(mtos or [])
    steps = [(int(round((float(m["time"]) - t_start) / dt)), m) for m in mt]
    cum = np.eye(dim * dim, dtype=complex)
    dm = np.empty((n, dim * dim, dim * dim), dtype=complex)
    for k in range(n):
        for s, m in steps:
            if s == k:
                cum = _superop(opgrammar.to_matrix(m["operator"], dim), m.get("applyFrom", ""), dim) @ cum
        H = H0 + np.sin(0.7 * (t_start + (k + 0.5) * dt)) * H1
        L = -1j * (np.kron(H, I) - np.kron(I, H.T))
        for Lk in Ls:
            LdL = Lk.conj().T @ Lk
            L = L + np.kron(Lk, Lk.conj()) - 0.5 * np.kron(LdL, I) - 0.5 * np.kron(I, LdL.T)
        cum = sla.expm(L * dt) @ cum
        dm[k] = cum
    return dm


def fake_system_dm(t_start, t_end, *pulses, dt=0.1, multitime_op=None, output_ops=[], trajectories=None,
                   calc_dynmap=False, fake_dim=2, **kw):
    """fake_system plus calc_dynmap=True -> ([t, outputs...], dm) from fake_dynmaps"""
    if not calc_dynmap:
        return fake_system(t_start, t_end, *pulses, dt=dt, multitime_op=multitime_op, output_ops=output_ops,
                           trajectories=trajectories, **kw)
    res = _run(t_start, t_end, dt, multitime_op, output_ops)
    return res, fake_dynmaps(t_start, t_end, dt, multitime_op, fake_dim)
