"""The blocked CPU port (oracle/pqd_oracle_blk.c, bench.py's CPU baseline) against the plain oracle
(oracle/pqd_oracle.c): same trajectories, MTOs of every kind before/after the outputs, several MTOs at one step,
ragged windows and lengths, partial blocks, with and without a PT, several systems."""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import pt as ptmod
from pyaceqd_amd.engine import MTO, Trajectories

from . import helpers as H


def _workload(N, n_steps, seed):
    rng = np.random.default_rng(seed)
    n_traj = 11
    begins = rng.integers(0, n_steps // 2, n_traj)
    ends = np.minimum(n_steps, begins + rng.integers(1, n_steps, n_traj))
    ends[0] = n_steps
    ends[1] = begins[1]  # a one-point window
    mtos = []
    for t in range(n_traj):
        for _ in range(int(rng.integers(0, 4))):
            step = int(rng.integers(0, ends[t] + 1))
            A = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
            mtos.append(MTO(t, step, bool(rng.integers(0, 2)), int(rng.integers(0, 3)), 0.5 * A))
    mtos.append(MTO(2, 3, False, 1, H.ketbra(N, 1, 0)))   # two at one step, list order matters
    mtos.append(MTO(2, 3, False, 2, H.ketbra(N, 0, 1)))
    rng.shuffle(mtos)
    return Trajectories(begins, ends, mtos), n_traj


def _cmp(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape
        assert np.max(np.abs(x - y)) <= 1e-12 * max(1.0, np.max(np.abs(y)))


@pytest.mark.parametrize("N,chi,bt", [(2, 8, 4), (3, 16, 8), (4, 16, 3), (4, 1, 8), (6, 8, 8)])
def test_blocked_port_matches_oracle(N, chi, bt):
    n_steps = 24
    sysd, grid = H.random_system(N, n_steps=n_steps, seed=3 * N + chi)
    tr, _ = _workload(N, n_steps, seed=N * 100 + chi)
    pt = None if chi == 1 else ptmod.random_pt(N, chi, D=N * N, n_slices=9, seed=N, eps=0.1)
    rho0 = H.random_rho(N)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, N - 1, 0), H.random_rho(N, seed=5)]
    ref = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=2)
    got = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=3, blocked=bt)
    _cmp(got, ref)


def test_blocked_port_several_systems():
    N, chi, n_steps = 4, 16, 20
    systems = [H.random_system(N, n_steps=n_steps, seed=s)[0] for s in range(3)]
    grid = H.random_system(N, n_steps=n_steps, seed=0)[1]
    tr, n_traj = _workload(N, n_steps, seed=9)
    tr.system = np.arange(n_traj) % 3
    pt = ptmod.random_pt(N, chi, D=16, n_slices=21, seed=2, eps=0.1)
    rho0 = H.ketbra(N, 0, 0)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 3)]
    _cmp(oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, blocked=8),
         oracle.propagate(systems, grid, rho0, ops, tr, pt=pt))
