"""Split groups carrying several trajectories (pt_msplit.hip, PQD_PATH_MSPLIT) vs the CPU oracle. GPU only.

A group of N^2 workgroups propagates TB trajectories, workgroup g owning PT row g of all of them; trajectory-steps
with MTOs use composite operators built on the device (evcomp_kernel). Covered: N = 3..6, chi = 32 / 64 (the PT
padded to them), TB = 1, 2, 3, 5 and the automatic choice, the XCD-grouped and the plain grid, MTOs of every kind
at step 0, mid-run and at a window's last step, applyBefore and applyAfter at one step, ragged windows and ends,
several systems in one group, a repeated slice (the slice row kept in registers), the C4 rank-shard shape, and the
batched fallback after a forced timeout. Tolerance 1e-11 relative, as every PT sweep test (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, Trajectories
from tests import helpers as H

pytestmark = pytest.mark.gpu
MSPLIT = "split groups, several trajectories per group"


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def cmp_lists(got, ref, tol):
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        assert rel(a, b) < tol, rel(a, b)


def mixed_trajectories(n_steps, N, n_traj, seed):
    """ragged windows and ends; MTO kinds 0/1/2 at step 0, mid-run, at the window's end, before and after at one
    step, two MTOs in one slot, and trajectories without MTOs"""
    rng = np.random.default_rng(seed)
    beg, end, mt = [], [], []
    for t in range(n_traj):
        e = int(rng.integers(n_steps // 2, n_steps + 1))
        b = int(rng.integers(0, e))
        beg.append(b)
        end.append(e)
        A = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
        C = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
        A, C = A / np.linalg.norm(A), C / np.linalg.norm(C)
        k = t % 6
        s = int(rng.integers(0, e + 1))
        if k == 0:
            mt += [MTO(t, s, False, 2, A), MTO(t, s, False, 1, C)]      # the two-time pair (right, left)
        elif k == 1:
            mt += [MTO(t, 0, True, 0, A)]                                # at step 0, before the first output
        elif k == 2:
            mt += [MTO(t, s, True, 1, A), MTO(t, s, False, 2, C)]       # before and after at one step
        elif k == 3:
            mt += [MTO(t, e, False, 0, A), MTO(t, max(0, e - 3), True, 2, C)]  # at the last step, and three before
        elif k == 4:
            mt += [MTO(t, s, False, 0, A), MTO(t, min(e, s + 1), False, 1, np.eye(N) * 0.5 + C)]
    return Trajectories(np.array(beg), np.array(end), mt)


@pytest.mark.parametrize("N,chi", [(3, 32), (3, 64), (4, 32), (4, 64), (5, 32), (6, 32), (6, 64)])
@pytest.mark.parametrize("tb", ["auto", "1", "3", "5"])
def test_msplit_vs_oracle(monkeypatch, N, chi, tb):
    monkeypatch.setenv("PQD_MSPLIT", "2")
    if tb != "auto":
        monkeypatch.setenv("PQD_MS_TB", tb)
    n_sys = 3
    systems = [H.random_system(N, n_steps=40, seed=60 + k)[0] for k in range(n_sys)]
    grid = Grid(0.0, 0.1, 40)
    n_traj = 21
    tr = mixed_trajectories(grid.n_steps, N, n_traj, seed=N + chi)
    tr.system = np.array([k % n_sys for k in range(n_traj)])
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=9, seed=chi + N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    path, bt, fb = plan.info()
    assert path == MSPLIT and fb == 0
    if tb != "auto":
        assert bt >= int(tb)  # raised where the device cannot hold the groups (N = 6: 21 trajectories need TB >= 3)
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("xcd", ["0", "1"])
@pytest.mark.parametrize("n_traj", [20, 32, 100])
def test_msplit_auto_bench_shape(monkeypatch, xcd, n_traj):
    """the C4 sweep shape at reduced length (bench.build_workload: MTO pair at t1, window [t1, t1 + n_tau], a repeated
    slice after 410 initial ones is not reached here, so a short n_init is used): auto mode takes the multi-trajectory
    groups past the single-trajectory capacity; vs the oracle"""
    import bench
    monkeypatch.setenv("PQD_SPLIT_XCD", xcd)
    systems, grid, _, rho0, ops, tr = bench.build_workload(n_traj, 300, 64, make_pt=False)
    pt = ptmod.synthetic_pt(np.diag([0, 1, 1, 2]).astype(complex), chi=64, n_init=12, n_rep=1, seed=5, eps=0.05,
                            dt=grid.dt)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_msplit_matches_batched_at_c4_shard_length(monkeypatch):
    """one rank's C4 shard (32 t1 points, MTO pair at t1, 10,000 tau steps, chi = 64, bench PT) on multi-trajectory
    groups equals the batched kernel's run at full length (both vs each other at 1e-10: 10,255 steps of rounding)"""
    import bench
    systems, grid, pt, rho0, ops, tr = bench.build_workload(32, 10000, 64, t1_offset=96)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    monkeypatch.setenv("PQD_SPLIT", "0")
    ref = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    ref.execute()
    cmp_lists(got, ref.download(), 1e-10)


@pytest.mark.parametrize("N,n_traj", [(3, 1), (4, 1), (4, 7)])
def test_msplit_chi128_vs_oracle(N, n_traj):
    """chi = 128 (a generated PT's bond cap at N <= 4, which the single-trajectory split kernel does not take): auto
    mode runs it on multi-trajectory split groups of one PT row per workgroup (a chi = 128 single
    run on the split path), vs the oracle"""
    systems = [H.random_system(N, n_steps=30, seed=80 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 30)
    tr = mixed_trajectories(grid.n_steps, N, n_traj, seed=N + 128)
    tr.system = np.array([k % 2 for k in range(n_traj)])
    pt = ptmod.random_pt(N, 100, D=min(N * N, 9), n_slices=7, seed=N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_msplit_timeout_falls_back_to_batched(monkeypatch):
    """PQD_SPLIT_SPIN=0: every wait for a peer times out; the plan re-runs the sweep on the batched kernel"""
    N, chi = 4, 64
    monkeypatch.setenv("PQD_MSPLIT", "2")
    monkeypatch.setenv("PQD_SPLIT_SPIN", "0")
    sysd, grid = H.random_system(N, n_steps=30, seed=8)
    tr = mixed_trajectories(30, N, 24, seed=4)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=6, seed=9, eps=0.1)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 2, 0)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    assert plan.info()[0] == MSPLIT
    plan.execute()
    got = plan.download()
    assert plan.info()[2] == 1 and plan.info()[0] == "batched lock-step sweep"
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_msplit_repeated_executes_and_rebuild(monkeypatch):
    """executing a plan twice (free propagators and composites rebuilt) gives identical outputs; executing without
    the rebuild keeps them too"""
    N, chi = 4, 64
    monkeypatch.setenv("PQD_MSPLIT", "2")
    sysd, grid = H.random_system(N, n_steps=25, seed=18)
    tr = mixed_trajectories(25, N, 40, seed=6)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=5, seed=3, eps=0.1)
    ops = [H.ketbra(N, 1, 1)]
    plan = engine.Plan(sysd, grid, H.random_rho(N), ops, tr, pt=pt)
    plan.execute()
    a = [x.copy() for x in plan.download()]
    plan.execute()
    b = plan.download()
    plan.execute(rebuild_free=False)
    c = plan.download()
    for x, y, z in zip(a, b, c):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)


@pytest.mark.parametrize("l2", ["1", "0"])
def test_msplit_exchange_store_flavours(monkeypatch, l2):
    """XCD-grouped grid: exchange stores that keep their L2 lines (default, the group's placement on one XCD checked
    at its first poll) and sc1 stores (PQD_MS_L2=0); both vs the oracle, no fallback"""
    monkeypatch.setenv("PQD_MSPLIT", "2")
    monkeypatch.setenv("PQD_MS_L2", l2)
    N, chi = 4, 64
    sysd, grid = H.random_system(N, n_steps=40, seed=21)
    tr = mixed_trajectories(40, N, 48, seed=12)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=7, seed=4, eps=0.12)
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 2, 0)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_msplit_spread_group_reruns_with_sc1_stores(monkeypatch):
    """PQD_ABLATE=512: workgroup 0 of every group reports another XCD, so the first poll finds the group spread; the
    launch ends before its first gather and the plan re-runs it with sc1 exchange stores (one fallback, still on split
    groups), vs the oracle"""
    monkeypatch.setenv("PQD_MSPLIT", "2")
    monkeypatch.setenv("PQD_ABLATE", "512")
    N, chi = 4, 64
    sysd, grid = H.random_system(N, n_steps=30, seed=22)
    tr = mixed_trajectories(30, N, 40, seed=13)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=6, seed=5, eps=0.1)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 3, 1)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 1
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)
    plan.execute()  # stays on sc1 stores: no further fallback
    cmp_lists(plan.download(), got, 1e-15)
    assert plan.info()[2] == 1


@pytest.mark.parametrize("N,chi", [(3, 32), (4, 64), (5, 32), (6, 64)])
@pytest.mark.parametrize("ptm", ["0", "1"])
@pytest.mark.parametrize("tb", ["1", "5", "8", "12", "16"])
def test_msplit_pt_on_valu_and_matrix_cores(monkeypatch, N, chi, ptm, tb):
    """the PT contraction on the FP64 VALU (DPP row broadcast) and on the matrix cores (3M 4x4x4_4b row blocks,
    PQD_MS_PTM), with partial row blocks (TB = 1, 5) and inactive slots, up to the 16 trajectories per group auto mode
    takes (two gather chunks per half, two row-block passes), vs the oracle"""
    monkeypatch.setenv("PQD_MSPLIT", "2")
    monkeypatch.setenv("PQD_MS_PTM", ptm)
    monkeypatch.setenv("PQD_MS_TB", tb)
    systems = [H.random_system(N, n_steps=36, seed=90 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 36)
    tr = mixed_trajectories(grid.n_steps, N, 19, seed=N + 7 * chi)
    tr.system = np.array([k % 2 for k in range(19)])
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=8, seed=chi + 3 * N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("N,n_traj,chi", [(2, 1, 200), (2, 9, 256), (3, 4, 160), (4, 1, 256), (4, 6, 180)])
def test_msplit_chi256_vs_oracle(N, n_traj, chi):
    """bonds past 128 (padded to 256: the slice rows streamed from L2 through the matrix-core PT, one PT row per
    workgroup of 1,024 threads) for the two-level system (N2 = 4, the only path that holds it), N = 3 and the biexciton,
    single and several trajectories per group, MTOs, vs the oracle (a path that holds a bond the
    generator's cap would otherwise cut)"""
    systems = [H.random_system(N, n_steps=24, seed=70 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 24)
    tr = mixed_trajectories(grid.n_steps, N, n_traj, seed=N + chi)
    tr.system = np.array([k % 2 for k in range(n_traj)])
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=5, seed=N + chi, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == MSPLIT and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_chi256_batch_beyond_one_launch_is_refused():
    """chi = 256 has no batched fallback: a batch the groups cannot hold in one launch is refused at plan creation"""
    N = 4
    sysd, grid = H.random_system(N, n_steps=8, seed=3)
    tr = Trajectories(np.zeros(300, dtype=int), np.full(300, 8))
    pt = ptmod.random_pt(N, 256, D=9, n_slices=2, seed=1, eps=0.1)
    with pytest.raises(Exception, match="chi 256"):
        engine.Plan(sysd, grid, H.random_rho(N), [H.ketbra(N, 1, 1)], tr, pt=pt)
