"""Known-answer tests and invariants that pin the PT-propagator oracle (the reference delegates this arithmetic to
the absent ACE binary, so parity with ACE itself is unpinned: SURVEY.md §8c)."""
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import oracle
from pyaceqd_amd import pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, System
from tests import helpers as H


def test_expm_matches_scipy():
    rng = np.random.default_rng(3)
    for n, s in [(4, 0.1), (16, 1.0), (36, 3.0), (9, 40.0)]:
        A = s * (rng.normal(size=(n, n)) + 1j * rng.normal(size=(n, n))) / np.sqrt(n)
        E = oracle.expm(A)
        R = sla.expm(A)
        assert np.max(np.abs(E - R)) / np.max(np.abs(R)) < 1e-12


def test_free_propagators_match_numpy_restatement():
    for N, n_sub in [(2, 1), (3, 2), (4, 1)]:
        sysd, grid = H.random_system(N, n_steps=6, n_sub=n_sub, seed=N)
        M = oracle.free_propagators(sysd, grid)
        R = H.numpy_free_props(sysd, grid)
        assert np.max(np.abs(M - R)) < 1e-12


@pytest.mark.parametrize("with_pt", [False, True])
def test_propagate_matches_numpy_restatement(with_pt):
    N = 3
    sysd, grid = H.random_system(N, n_steps=12, seed=7)
    rho0 = H.random_rho(N)
    out_ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 2), np.eye(N)]
    mt = [MTO(0, 3, False, 1, H.ketbra(N, 1, 0)), MTO(0, 3, False, 2, H.ketbra(N, 0, 1)),
          MTO(1, 0, True, 0, H.ketbra(N, 2, 0) + H.ketbra(N, 0, 2)), MTO(1, 5, True, 2, np.diag([1, 2, 3.0]))]
    tr = H.simple_traj(grid.n_steps, mt, n_traj=2, begins=[0, 2], ends=[12, 9])
    pt = ptmod.random_pt(N, 4, D=5, n_slices=3, seed=2) if with_pt else None
    a = oracle.propagate(sysd, grid, rho0, out_ops, tr, pt=pt)
    b = H.numpy_propagate(sysd, grid, rho0, out_ops, tr, pt=pt)
    for x, y in zip(a, b):
        assert x.shape == y.shape
        assert np.max(np.abs(x - y)) / np.max(np.abs(y)) < 1e-11


@pytest.mark.parametrize("area", [0.5, 1.0, 2.0, 3.3])
def test_kat_rabi_rotation(area):
    """resonant unchirped Gaussian of area pi*e0: rho_11(te) = sin^2(pi e0 / 2)"""
    sysd, grid = H.rabi_system(area_pi=area, tau=1.5, t0=10.0, dt=0.02, te=20.0)
    out = oracle.propagate(sysd, grid, H.ketbra(2, 0, 0), [H.ketbra(2, 1, 1)], H.simple_traj(grid.n_steps))[0]
    assert abs(out[-1, 0].real - np.sin(np.pi * area / 2) ** 2) < 1e-8


def test_kat_decay():
    """add_Lindblad gamma {|0><1|}: x(t) = exp(-gamma t)"""
    g = 0.37
    sysd = System(dim=2, H0=np.diag([0.0, 1.3]), lindblad=[(g, H.ketbra(2, 0, 1))])
    grid = Grid(0.0, 0.1, 200)
    out = oracle.propagate(sysd, grid, H.ketbra(2, 1, 1), [H.ketbra(2, 1, 1), np.eye(2)], H.simple_traj(200))[0]
    t = grid.times
    assert np.max(np.abs(out[:, 0] - np.exp(-g * t))) < 1e-12
    assert np.max(np.abs(out[:, 1] - 1.0)) < 1e-12  # trace preservation


def test_kat_cw_rabi():
    """constant drive f: rho_11 = sin^2(Omega t / 2), Omega = pi f"""
    f0, dt, n = 0.2, 0.05, 400
    ds = dt / 4
    X = -0.5 * np.pi * H.hbar * H.ketbra(2, 1, 0)
    sysd = System(dim=2, H0=np.zeros((2, 2)), channels=[(X, np.full(4 * n + 1, f0, dtype=complex))], sample_dt=ds)
    out = oracle.propagate(sysd, Grid(0.0, dt, n), H.ketbra(2, 0, 0), [H.ketbra(2, 1, 1)], H.simple_traj(n))[0]
    t = dt * np.arange(n + 1)
    assert np.max(np.abs(out[:, 0].real - np.sin(np.pi * f0 * t / 2) ** 2)) < 1e-12


def test_pt_structured_invariant():
    """a PT whose bond channel 0 is decoupled (closure = bond0 = e_0) must reproduce the bare dynamics"""
    N = 4
    sysd, grid = H.random_system(N, n_steps=15, seed=11)
    boson = np.diag([0, 1, 1, 2.0])
    pt = ptmod.synthetic_pt(boson, chi=8, n_init=4, n_rep=3, seed=3)
    rho0 = H.random_rho(N)
    ops = [H.ketbra(N, k, k) for k in range(N)] + [H.ketbra(N, 0, 3)]
    tr = H.simple_traj(grid.n_steps)
    a = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt)[0]
    b = oracle.propagate(sysd, grid, rho0, ops, tr)[0]
    assert np.max(np.abs(a - b)) < 1e-13


def test_pt_markov_dephasing_equals_lindblad():
    """pure dephasing encoded in a chi=1 PT == Lindblad dephasing (commuting case: diagonal H, decay)"""
    N, g, dt = 3, 0.4, 0.1
    A = np.diag([0.0, 1.0, 2.0])
    H0 = np.diag([0.0, 0.7, -0.2])
    base = System(dim=N, H0=H0, lindblad=[(0.1, H.ketbra(N, 0, 1))])
    lind = System(dim=N, H0=H0, lindblad=[(0.1, H.ketbra(N, 0, 1)), (g, A)])
    grid = Grid(0.0, dt, 60)
    rho0 = H.random_rho(N, seed=4)
    ops = [H.ketbra(N, i, j) for i in range(N) for j in range(N)]
    tr = H.simple_traj(60)
    pt = ptmod.markov_dephasing_pt(A, g, dt)
    a = oracle.propagate(base, grid, rho0, ops, tr, pt=pt)[0]
    b = oracle.propagate(lind, grid, rho0, ops, tr)[0]
    assert np.max(np.abs(a - b)) < 1e-13


def test_mto_timing_semantics():
    """applyBefore false: visible one step after `time`; true: visible at `time` (general_system.py:283-285)"""
    N = 2
    sysd = System(dim=N, H0=np.zeros((2, 2)))
    grid = Grid(0.0, 0.1, 10)
    flip = H.ketbra(2, 1, 0) + H.ketbra(2, 0, 1)
    for before, first in [(False, 5), (True, 4)]:
        tr = H.simple_traj(10, [MTO(0, 4, before, 0, flip)])
        out = oracle.propagate(sysd, grid, H.ketbra(2, 0, 0), [H.ketbra(2, 1, 1)], tr)[0][:, 0].real
        assert np.all(out[:first] == 0) and np.all(out[first:] == 1)
