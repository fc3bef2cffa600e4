"""Pulse windows (free_prop.hip free_win_kernel, pqd_common.h fw_M / fw_F / fw_W). GPU only.

A system's half steps outside [first, last] half step with a non-zero pulse sample are not stored; the quad and no-PT
kernels read the system's idle operators there (Midle, Fidle = Midle Midle, Widle = ovec . Midle, built with the
storing kernels' own arithmetic). Plans on the batched sweep (or with a trunk pre-pass, or split groups that may fall
back to it) build every half step, and a window that leaves out less than a tenth is dropped (test_window_selection).
The outputs must be bit-identical to storing every half step (PQD_WIN=0) on every path —
quads, the batched sweep, split groups, the no-PT kernel, shared trunks — with several systems of different windows
in one plan (pulse early, late, two pulses with an idle gap inside the window, never, always), MTOs inside and
outside the windows, and fused and unfused half steps; and within 1e-11 of the CPU oracle."""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, pt as ptmod
from pyaceqd_amd.engine import Grid, Trajectories
from tests import helpers as H
from tests.test_gpu_parity import _traj, cmp_lists

pytestmark = pytest.mark.gpu

# pulse support per system, as fractions of the sample range
SEGMENTS = [[(0.10, 0.25)], [(0.60, 0.80)], [(0.05, 0.15), (0.55, 0.65)], [], [(0.0, 1.0)]]


def _windowed_systems(N, n_steps, n_sub=1, seed=0):
    out = []
    for k, segs in enumerate(SEGMENTS):
        sysd, grid = H.random_system(N, n_steps=n_steps, n_sub=n_sub, seed=seed + k)
        chans = []
        for X, f in sysd.channels:
            f = np.array(f)
            keep = np.zeros(len(f), bool)
            for a, b in segs:
                keep[int(a * len(f)):int(b * len(f))] = True
            f[~keep] = 0.0
            chans.append((X, f))
        sysd.channels = chans
        out.append(sysd)
    return out, grid


def _both(monkeypatch, systems, grid, rho0, ops, tr, pt):
    res = []
    for w in ("1", "0"):
        monkeypatch.setenv("PQD_WIN", w)
        plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
        plan.execute()
        res.append((plan.download(), plan.info()[0]))
    (a, pa), (b, pb) = res
    assert pa == pb
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    return a, pa


@pytest.mark.parametrize("case", ["quad", "quad_unfused", "batched", "batched_unfused", "split", "nopt", "n6"])
def test_windows_bit_identical_and_oracle(monkeypatch, case):
    N = {"batched": 3, "batched_unfused": 4, "split": 4, "n6": 6}.get(case, 2)
    chi = {"nopt": None, "split": 32, "n6": 16}.get(case, 32 if N == 2 else 16)
    monkeypatch.setenv("PQD_FUSE", "0" if case.endswith("unfused") else "1")
    monkeypatch.setenv("PQD_SPLIT", "2" if case == "split" else "0")
    n_steps = 60
    systems, grid = _windowed_systems(N, n_steps, seed=10 * N)
    n_traj = 3 if case == "split" else 17
    tr = _traj(n_steps, N, n_traj, seed=N + 5)
    tr.system = np.array([k % len(systems) for k in range(n_traj)])
    pt = None if chi is None else ptmod.random_pt(N, chi, D=min(N * N, 4), n_slices=7, seed=chi, eps=0.1)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), H.random_rho(N, seed=4)]
    rho0 = H.random_rho(N)
    got, path = _both(monkeypatch, systems, grid, rho0, ops, tr, pt)
    expect = {"quad": "register-resident TLS quads", "quad_unfused": "register-resident TLS quads",
              "split": "split groups", "nopt": "no PT (one wave per trajectory)"}.get(case, "batched lock-step sweep")
    assert path == expect
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("N", [2, 4])
@pytest.mark.parametrize("mode", ["branch", "trunk"])
def test_windows_shared_trunks(monkeypatch, N, mode):
    """G2-shaped sweeps (trajectories from step 0 with their MTO at t1) over windowed systems: in-workgroup chains
    and the trunk pre-pass read the idle operators too"""
    monkeypatch.setenv("PQD_SPLIT", "0")
    monkeypatch.setenv("PQD_BRANCH", "1")
    monkeypatch.setenv("PQD_TRUNK", "1" if mode == "trunk" else "0")
    n_steps = 80
    systems, grid = _windowed_systems(N, n_steps, seed=3)
    from pyaceqd_amd.engine import MTO
    beg, end, mtos = [], [], []
    for k in range(24):
        t1 = 3 * k
        beg.append(t1)
        end.append(min(n_steps, t1 + 30))
        mtos.append(MTO(k, t1, k % 2 == 0, 1, H.ketbra(N, 1, 0) + 0.1 * np.eye(N)))
    tr = Trajectories(np.array(beg), np.array(end), mtos)  # every trajectory runs from step 0
    tr.system = np.array([k % len(systems) for k in range(24)])
    pt = ptmod.random_pt(N, 16, D=4, n_slices=9, seed=5, eps=0.1)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)]
    rho0 = H.ketbra(N, 0, 0)
    got, _ = _both(monkeypatch, systems, grid, rho0, ops, tr, pt)
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("N,n_sub", [(2, 2), (4, 1)])
def test_windows_long_idle_scan(monkeypatch, N, n_sub):
    """16 systems, pulse in the first fifth of 2,000 steps (many window chunks per system): bit-identical to storing
    every half step, and the dense free_propagators export still stores every half step"""
    n_steps = 2000
    systems = []
    for k in range(16):
        sysd, grid = H.random_system(N, n_steps=n_steps, n_sub=n_sub, seed=k)
        chans = []
        for X, f in sysd.channels:
            f = np.array(f)
            f[len(f) // 5:] = 0.0
            chans.append((X, f))
        sysd.channels = chans
        systems.append(sysd)
    dense = engine.free_propagators(systems[0], grid)
    assert np.array_equal(dense[-1], dense[-3])  # idle tail: copies of one matrix
    tr = Trajectories(np.zeros(16, int), np.full(16, n_steps))
    tr.system = np.arange(16)
    pt = ptmod.random_pt(N, 16, D=4, n_slices=9, seed=1, eps=0.1)
    ops = [H.ketbra(N, 1, 1)]
    rho0 = H.ketbra(N, 0, 0)
    _both(monkeypatch, systems, grid, rho0, ops, tr, pt)


@pytest.mark.parametrize("case,win,expect", [("quad", "1", True), ("nopt", "1", True), ("batched", "1", False),
                                             ("batched", "2", False), ("quad_full", "1", False),
                                             ("quad_full", "2", True), ("quad", "0", False)])
def test_window_selection(monkeypatch, case, win, expect):
    """windows only where every kernel of the plan reads through them (quad, no-PT), only when they leave out at least
    a tenth of the half steps unless forced (PQD_WIN=2), never with PQD_WIN=0"""
    monkeypatch.setenv("PQD_WIN", win)
    N = 3 if case == "batched" else 2
    n_steps = 60
    systems, grid = _windowed_systems(N, n_steps, seed=7)
    systems = [systems[4]] if case == "quad_full" else [systems[0], systems[1]]  # whole run driven / short pulses
    pt = None if case == "nopt" else ptmod.random_pt(N, 16, D=min(N * N, 4), n_slices=7, seed=3, eps=0.1)
    tr = Trajectories(np.zeros(8, dtype=int), np.full(8, n_steps), system=np.arange(8) % len(systems))
    plan = engine.Plan(systems, grid, H.random_rho(N), [H.ketbra(N, 0, 0)], tr, pt=pt)
    assert plan.windows() == expect
