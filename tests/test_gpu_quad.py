"""The register-resident two-level-system sweep (pt_quad.hip, PQD_PATH_QUAD) vs the CPU oracle. GPU only.

Covers what the kernel handles lane by lane: four trajectories per quad with their own systems, windows, MTO
events (every kind, before/after, at step 0 and at the last step), fused and unfused half steps, shared-trunk
activation (in-quad chains and trunk checkpoints), partial quads, 1 and 2 quads per workgroup, more than four output
operators, and bond dimensions padded to 16 and 32. Tolerance 1e-11 relative, as for every PT sweep
(test_gpu_parity.py)."""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, Trajectories
from tests import helpers as H
from tests.test_gpu_parity import _traj, cmp_lists

pytestmark = pytest.mark.gpu


def _run(systems, grid, rho0, ops, tr, pt):
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    return got, plan.info()[0]


@pytest.mark.parametrize("chi", [8, 16, 32, 64])
@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("qpw", ["1", "2"])
@pytest.mark.parametrize("qcg", ["1", "2", "4"])
def test_quad_vs_oracle(monkeypatch, chi, fuse, qpw, qcg):
    monkeypatch.setenv("PQD_FUSE", fuse)
    monkeypatch.setenv("PQD_QPW", qpw)
    monkeypatch.setenv("PQD_QCG", qcg)
    monkeypatch.setenv("PQD_SPLIT", "0")
    if chi == 64:
        monkeypatch.setenv("PQD_QUAD", "2")  # chi = 64 quads are opt-in
    N = 2
    systems = [H.random_system(N, n_steps=40, seed=60 + k)[0] for k in range(3)]
    grid = Grid(0.0, 0.1, 40)
    tr = _traj(grid.n_steps, N, 23, seed=chi + 7)
    tr.system = np.array([k % 3 for k in range(23)])
    pt = ptmod.random_pt(N, chi, D=4, n_slices=11, seed=chi, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N), H.ketbra(N, 0, 1), H.ketbra(N, 1, 1),
           H.random_rho(N, seed=3)]
    rho0 = H.random_rho(N)
    got, path = _run(systems, grid, rho0, ops, tr, pt)
    assert path == "register-resident TLS quads"
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("n_traj", [1, 3, 4, 5, 9])
def test_quad_partial_quads(monkeypatch, n_traj):
    monkeypatch.setenv("PQD_SPLIT", "0")
    N = 2
    sysd, grid = H.random_system(N, n_steps=30, seed=n_traj)
    tr = _traj(grid.n_steps, N, n_traj, seed=n_traj + 100)
    pt = ptmod.random_pt(N, 32, D=4, n_slices=5, seed=4, eps=0.1)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)]
    rho0 = H.ketbra(N, 0, 0)
    got, path = _run(sysd, grid, rho0, ops, tr, pt)
    assert path == "register-resident TLS quads"
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt), 1e-11)


def _g2_sweep(n_t1, n_tau, seed):
    """a TLS two-time sweep shaped like the reference callers: every trajectory runs from step 0, MTOs at t1
    (correlations.py:155-169), so trajectories of one system share their trunk up to their branch step"""
    N = 2
    sysd, grid = H.random_system(N, n_steps=2 * n_t1 + n_tau, seed=seed)
    A, C = H.ketbra(N, 1, 0), H.ketbra(N, 0, 1)
    mtos, beg, end = [], [], []
    for t1 in range(n_t1):
        t = len(beg)
        mtos += [MTO(t, 2 * t1, False, 2, A), MTO(t, 2 * t1, False, 1, C)]
        beg.append(2 * t1)
        end.append(2 * t1 + n_tau)
    return sysd, grid, Trajectories(np.array(beg), np.array(end), mtos)


@pytest.mark.parametrize("mode", ["branch", "trunk", "none"])
@pytest.mark.parametrize("qcg", ["1", "2", "4"])
def test_quad_shared_trunks(monkeypatch, mode, qcg):
    monkeypatch.setenv("PQD_QCG", qcg)
    monkeypatch.setenv("PQD_SPLIT", "0")
    monkeypatch.setenv("PQD_BRANCH", "0" if mode == "none" else "1")
    monkeypatch.setenv("PQD_TRUNK", "1" if mode == "trunk" else "0")
    sysd, grid, tr = _g2_sweep(13, 20, seed=8)
    pt = ptmod.random_pt(2, 32, D=4, n_slices=9, seed=8, eps=0.1)
    ops = [H.ketbra(2, 1, 1), H.ketbra(2, 0, 1)]
    rho0 = H.ketbra(2, 0, 0)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == "register-resident TLS quads"
    if mode != "none":
        assert plan.traj_steps() < int(np.sum(tr.out_end + 1))
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt), 1e-11)


def test_quad_matches_batched_kernel(monkeypatch):
    """the same C2-shaped scan (one system per trajectory) on the quad kernel and on the BT = 8 batched kernel"""
    monkeypatch.setenv("PQD_SPLIT", "0")
    N = 2
    systems = [H.random_system(N, n_steps=200, seed=200 + k)[0] for k in range(16)]
    grid = Grid(0.0, 0.1, 200)
    tr = Trajectories(np.zeros(16, int), np.full(16, 200))
    tr.system = np.arange(16)
    pt = ptmod.random_pt(N, 32, D=4, n_slices=60, seed=2, eps=0.1)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)]
    rho0 = H.ketbra(N, 0, 0)
    a, path = _run(systems, grid, rho0, ops, tr, pt)
    assert path == "register-resident TLS quads"
    monkeypatch.setenv("PQD_QUAD", "0")
    b, path = _run(systems, grid, rho0, ops, tr, pt)
    assert path == "batched lock-step sweep"
    cmp_lists(a, b, 1e-11)
