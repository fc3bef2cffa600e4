"""Shared builders for tests: small systems, trajectories and a pure-numpy restatement of the
propagation semantics (used only for tiny sizes, as an independent cross-check of the C oracle)."""
import numpy as np
import scipy.linalg as sla

from pyaceqd_amd.engine import Grid, MTO, System, Trajectories
from pyaceqd_amd.constants import hbar


def ketbra(N, a, b):
    m = np.zeros((N, N), dtype=complex)
    m[a, b] = 1
    return m


def random_system(N, n_chan=2, n_lind=2, seed=0, n_steps=20, dt=0.1, ta=0.0, n_sub=1):
    rng = np.random.default_rng(seed)
    H = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
    H = 0.5 * (H + H.conj().T)
    lind = [(0.05 * (k + 1), rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))) for k in range(n_lind)]
    ds = dt / (4 * n_sub)
    ns = 4 * n_sub * n_steps + 1
    tt = ta + ds * np.arange(ns)
    chans = []
    for c in range(n_chan):
        X = 0.5 * (rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N)))
        f = np.exp(-((tt - tt.mean()) / (0.3 * (tt[-1] - tt[0] + 1e-9))) ** 2) * np.exp(1j * (c + 1) * tt)
        chans.append((X, f))
    sysd = System(dim=N, H0=H, lindblad=lind, channels=chans, sample_t0=ta, sample_dt=ds)
    return sysd, Grid(ta, dt, n_steps, n_sub)


def random_rho(N, seed=1):
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
    r = A @ A.conj().T
    return r / np.trace(r)


def numpy_liouvillian(sysd, t):
    N = sysd.dim
    I = np.eye(N)
    H = np.array(sysd.H0, dtype=complex)
    u = (t - sysd.sample_t0) / sysd.sample_dt
    for X, f in sysd.channels:
        ns = len(f)
        if u <= 0:
            fv = f[0]
        elif u >= ns - 1:
            fv = f[-1]
        else:
            k = int(np.floor(u))
            fv = f[k] + (u - k) * (f[k + 1] - f[k])
        H = H + fv * X + np.conj(fv) * X.conj().T
    L = -1j / sysd.hbar * (np.kron(H, I) - np.kron(I, H.T))
    for g, Lk in sysd.lindblad:
        LdL = Lk.conj().T @ Lk
        L = L + g * (np.kron(Lk, Lk.conj()) - 0.5 * np.kron(LdL, I) - 0.5 * np.kron(I, LdL.T))
    return L


def numpy_free_props(sysd, grid):
    out = []
    w = 0.5 * grid.dt / grid.n_sub
    for n in range(grid.n_steps):
        for h in range(2):
            M = np.eye(sysd.dim ** 2, dtype=complex)
            for j in range(grid.n_sub):
                t = grid.ta + n * grid.dt + h * 0.5 * grid.dt + (j + 0.5) * w
                M = sla.expm(numpy_liouvillian(sysd, t) * w) @ M
            out.append(M)
    return np.array(out)


def numpy_propagate(sysd, grid, rho0, out_ops, traj, pt=None):
    """direct restatement with superoperators and einsum (small sizes only)"""
    N = sysd.dim
    N2 = N * N
    M = numpy_free_props(sysd, grid)
    chi = pt.chi if pt is not None else 1
    res = []
    for t in range(traj.n_traj):
        st = np.outer(np.asarray(rho0).reshape(N2), pt.bond0 if pt is not None else [1.0]).astype(complex)
        b, e = int(traj.out_begin[t]), int(traj.out_end[t])
        rows = []
        mt = [m for m in traj.mtos if m.traj == t]

        def apply(m, st):
            A = np.asarray(m.op)
            S = {0: np.kron(A, A.conj()), 1: np.kron(A, np.eye(N)), 2: np.kron(np.eye(N), A.T)}[m.kind]
            return S @ st
        sched = pt.schedule(max(1, grid.n_steps)) if pt is not None else None
        for n in range(e + 1):
            for m in mt:
                if m.step == n and m.before:
                    st = apply(m, st)
            if n >= b:
                c = (pt.closure0 if n == 0 else pt.closure[sched[n - 1]]) if pt is not None else np.ones(1)
                r = st @ c
                rows.append([np.trace(np.asarray(O) @ r.reshape(N, N)) for O in out_ops])
            for m in mt:
                if m.step == n and not m.before:
                    st = apply(m, st)
            if n == e:
                break
            st = M[2 * n] @ st
            if pt is not None:
                Qs = pt.Q[sched[n]]
                st = np.stack([st[a] @ Qs[pt.gmap[a]] for a in range(N2)])
            st = M[2 * n + 1] @ st
        res.append(np.array(rows))
    return res


def simple_traj(n_steps, mtos=(), n_traj=1, begins=None, ends=None):
    begins = np.zeros(n_traj, dtype=int) if begins is None else np.asarray(begins)
    ends = np.full(n_traj, n_steps) if ends is None else np.asarray(ends)
    return Trajectories(begins, ends, list(mtos))


def rabi_system(area_pi=1.0, tau=2.0, t0=10.0, gamma=0.0, dt=0.05, te=20.0):
    """resonant TLS driven by a unit-area Gaussian scaled to `area_pi` (units of pi): H = -pi hbar/2 (f s+ + h.c.)"""
    N = 2
    n_steps = int(round(te / dt))
    ds = dt / 4
    tt = ds * np.arange(4 * n_steps + 1)
    f = area_pi * np.exp(-0.5 * ((tt - t0) / tau) ** 2) / (np.sqrt(2 * np.pi) * tau)
    X = -0.5 * np.pi * hbar * ketbra(N, 1, 0)
    lind = [(gamma, ketbra(N, 0, 1))] if gamma else []
    return System(dim=2, H0=np.zeros((2, 2)), lindblad=lind, channels=[(X, f.astype(complex))], sample_t0=0.0,
                  sample_dt=ds), Grid(0.0, dt, n_steps, 1)
