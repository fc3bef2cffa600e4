"""Shared trunks in the lock-step sweep (DESIGN.md §4.1 "shared trunk"). GPU only.

Trajectories of one system that share a workgroup propagate their common MTO-free trunk once: a slot stays dormant
until its activation step, then copies the (state, fused flag) of an earlier slot. Every trajectory's outputs must
still be those of its own full run (the CPU oracle propagates every trajectory from step 0), for every MTO kind and
timing (applyBefore true/false, MTOs at step 0, several MTOs), output windows that open before the MTO, trajectories
without MTOs, multi-system workgroups, BT = 4 and 8, fused and unfused half steps, all PT contraction modes.
"""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, Trajectories
from tests import helpers as H

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def g2_reuse_shape(n_steps, n_t1, N, n_sys=1, seed=0, mixed=True):
    """pol_entanglement.G2_reuse / _ops_two_time shape: trajectory i gets its MTO pair at t1_i and runs to the end;
    `mixed` adds applyBefore MTOs, early windows, MTO-free and step-0 trajectories"""
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
    C = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
    A, C = A / np.linalg.norm(A), C / np.linalg.norm(C)
    beg, end, mtos, sysidx = [], [], [], []
    for i in range(n_t1):
        t1 = int(i * (n_steps - 2) / max(1, n_t1 - 1))
        t = len(beg)
        kind = i % 7 if mixed else 0
        if kind == 3:          # applyBefore MTO: acts before the output at t1
            mtos.append(MTO(t, max(t1, 1), True, 0, A))
        elif kind == 5:        # no MTO at all
            pass
        elif kind == 6:        # MTO at step 0
            mtos += [MTO(t, 0, False, 2, A), MTO(t, 0, False, 1, C)]
        else:
            mtos += [MTO(t, t1, False, 2, A), MTO(t, t1, False, 1, C)]
            if kind == 4:      # a second, later MTO
                mtos.append(MTO(t, min(n_steps, t1 + 3), False, 1, C))
        beg.append(max(0, t1 - 2) if kind == 2 else t1)   # kind 2: window opens before the MTO
        end.append(n_steps if kind != 1 else max(t1, n_steps - 4))
        sysidx.append(i % n_sys)
    return Trajectories(np.array(beg), np.array(end), mtos, system=np.array(sysidx) if n_sys > 1 else None)


@pytest.mark.parametrize("N,chi,bt", [(2, 32, "8"), (3, 16, "4"), (4, 64, "8"), (4, 64, "4"), (6, 32, "4")])
@pytest.mark.parametrize("fuse", ["0", "1"])
def test_branching_matches_full_runs(monkeypatch, N, chi, bt, fuse):
    monkeypatch.setenv("PQD_BT", bt)
    monkeypatch.setenv("PQD_FUSE", fuse)
    monkeypatch.setenv("PQD_SPLIT", "0")
    n_sys = 2
    systems = [H.random_system(N, n_steps=36, seed=20 + k)[0] for k in range(n_sys)]
    grid = Grid(0.0, 0.1, 36)
    tr = g2_reuse_shape(36, 29, N, n_sys=n_sys, seed=N + chi)
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=12, seed=chi + N, eps=0.12)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    monkeypatch.setenv("PQD_BRANCH", "1")
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    full = int(np.sum(tr.out_end + 1))
    assert plan.traj_steps() < full
    plan.execute()
    got = plan.download()
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        assert rel(a, b) < 1e-11, rel(a, b)
    monkeypatch.setenv("PQD_BRANCH", "0")
    plan0 = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    assert plan0.traj_steps() == full


@pytest.mark.parametrize("pt_mode", ["0", "1", "2", "3", "4", "5"])
def test_branching_all_pt_modes(monkeypatch, pt_mode):
    N, chi = 4, 32
    monkeypatch.setenv("PQD_PT_MODE", pt_mode)
    monkeypatch.setenv("PQD_BT", "4" if pt_mode == "0" else "8")
    monkeypatch.setenv("PQD_SPLIT", "0")
    sysd, grid = H.random_system(N, n_steps=30, seed=3)
    tr = g2_reuse_shape(30, 21, N, seed=9)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=8, seed=5, eps=0.12)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 2)]
    rho0 = H.random_rho(N)
    got = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    ref = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-11, rel(a, b)


def test_g2_reuse_shape_halves_executed_steps(monkeypatch):
    """every trajectory runs 0 -> n_end with its MTOs at t1 uniformly spread (the reference's G2_reuse shape):
    the shared trunks leave about half of the trajectory-steps"""
    N, chi, n_steps, n_t1 = 4, 16, 400, 256
    monkeypatch.setenv("PQD_SPLIT", "0")
    monkeypatch.setenv("PQD_BT", "8")
    sysd, grid = H.random_system(N, n_steps=n_steps, seed=4)
    tr = g2_reuse_shape(n_steps, n_t1, N, seed=2, mixed=False)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=20, seed=6, eps=0.1)
    ops = [H.ketbra(N, 1, 1)]
    rho0 = H.ketbra(N, 0, 0)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    full = int(np.sum(tr.out_end + 1))
    assert plan.traj_steps() < 0.6 * full
    plan.execute()
    got = plan.download()
    monkeypatch.setenv("PQD_BRANCH", "0")
    ref = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-12


# ------------------------------------------------------------------------------------------- trunk pre-pass
@pytest.mark.parametrize("N,chi,bt", [(2, 32, "8"), (3, 16, "4"), (4, 64, "8"), (4, 32, "4"), (6, 16, "4")])
def test_trunk_prepass_matches_full_runs(monkeypatch, N, chi, bt):
    """PQD_TRUNK=1: every slot starts at its branch step from a checkpoint of its system's trunk (split groups at
    N^2 >= 9, batched workgroups below)"""
    monkeypatch.setenv("PQD_BT", bt)
    monkeypatch.setenv("PQD_TRUNK", "1")
    n_sys = 3
    systems = [H.random_system(N, n_steps=36, seed=30 + k)[0] for k in range(n_sys)]
    grid = Grid(0.0, 0.1, 36)
    tr = g2_reuse_shape(36, 31, N, n_sys=n_sys, seed=N * chi)
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=12, seed=chi + 2 * N, eps=0.12)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[2] == 0
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        assert rel(a, b) < 1e-11, rel(a, b)


def test_trunk_prepass_split_timeout_falls_back(monkeypatch):
    N, chi = 4, 32
    monkeypatch.setenv("PQD_TRUNK", "1")
    monkeypatch.setenv("PQD_SPLIT_SPIN", "0")
    systems = [H.random_system(N, n_steps=40, seed=50 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 40)
    tr = g2_reuse_shape(40, 17, N, n_sys=2, seed=3)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=9, seed=8, eps=0.1)
    ops = [H.ketbra(N, 1, 1)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[2] == 1
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-11, rel(a, b)


@pytest.mark.parametrize("spin", ["default", "0"])
def test_trunk_prepass_in_consecutive_launches(monkeypatch, spin):
    """more six-level trunks than the device holds as co-resident split groups (8 trunks x 36 workgroups on 256
    CUs: 7 + 1 launches, pqd_host.cpp tk_chunk; the C5 tomography scan's shape). With PQD_SPLIT_SPIN=0 every wait
    for a peer times out and the pre-pass falls back to batched workgroups"""
    N, chi, n_sys = 6, 16, 8
    monkeypatch.setenv("PQD_TRUNK", "1")
    if spin == "0":
        monkeypatch.setenv("PQD_SPLIT_SPIN", "0")
    systems = [H.random_system(N, n_steps=30, seed=70 + k)[0] for k in range(n_sys)]
    grid = Grid(0.0, 0.1, 30)
    tr = g2_reuse_shape(30, 40, N, n_sys=n_sys, seed=11)
    pt = ptmod.random_pt(N, chi, D=9, n_slices=8, seed=12, eps=0.1)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 5, 0)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[2] == (1 if spin == "0" else 0)
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-11, rel(a, b)


def test_trunk_prepass_halves_g2_reuse_steps(monkeypatch):
    N, chi, n_steps, n_t1 = 4, 16, 400, 256
    monkeypatch.setenv("PQD_TRUNK", "1")
    sysd, grid = H.random_system(N, n_steps=n_steps, seed=4)
    tr = g2_reuse_shape(n_steps, n_t1, N, seed=2, mixed=False)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=20, seed=6, eps=0.1)
    ops = [H.ketbra(N, 1, 1)]
    rho0 = H.ketbra(N, 0, 0)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    full = int(np.sum(tr.out_end + 1))
    assert plan.traj_steps() < 0.51 * full
    plan.execute()
    got = plan.download()
    monkeypatch.setenv("PQD_BRANCH", "0")
    ref = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-12


def test_bench_shaped_workload_auto_trunk(monkeypatch):
    """the bench's two-time sweep shape (scan points x t1 grid, fixed tau window) at reduced size, auto policy"""
    import bench
    systems, grid, pt, rho0, ops, tr = bench.build_workload(24, 60, 32, scan=3)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-11, rel(a, b)
    assert plan.traj_steps() <= int(np.sum(tr.out_end + 1))
