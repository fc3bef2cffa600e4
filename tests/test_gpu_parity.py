"""HIP path (libpqd via the C-ABI) vs the CPU oracle and the reference's golden vectors. GPU only.

Tolerances: the FP64 kernels and the oracle do the same arithmetic in different summation orders;
relative differences stay at a few 1e-14 per step. Tests use 1e-11 (PT sweeps, with up to 1e2-step
error growth) and 1e-12 elsewhere — far below the north-star bar (1e-8 abs no-phonon, 1e-6 rel with
phonons)."""
import os

import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, System, Trajectories
from tests import helpers as H

pytestmark = pytest.mark.gpu
F = lambda maps: np.asfortranarray(np.asarray(maps).transpose(1, 2, 0))  # noqa: E731


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def cmp_lists(got, ref, tol):
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        assert rel(a, b) < tol, rel(a, b)


# --------------------------------------------------------------------------------- free propagators
@pytest.mark.parametrize("N,n_sub", [(2, 1), (3, 1), (4, 1), (4, 3), (5, 1), (6, 1), (6, 2)])
def test_free_propagators(N, n_sub):
    sysd, grid = H.random_system(N, n_steps=25, n_sub=n_sub, seed=N + 10 * n_sub)
    got = engine.free_propagators(sysd, grid)
    ref = oracle.free_propagators(sysd, grid)
    assert rel(got, ref) < 1e-12


# --------------------------------------------------------------------------------- sweeps
def _traj(n_steps, N, n_traj, seed):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, n_steps // 2, size=n_traj)
    e = np.minimum(n_steps, b + rng.integers(1, n_steps, size=n_traj))
    mt = []
    for t in range(n_traj):
        s = int(rng.integers(0, e[t] + 1))
        A = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
        mt.append(MTO(t, s, bool(rng.integers(0, 2)), int(rng.integers(0, 3)), A / np.linalg.norm(A)))
        if t % 2:
            mt.append(MTO(t, s, False, 1, np.eye(N) * 0.5 + A / np.linalg.norm(A)))
    return Trajectories(b, e, mt)


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("n_traj", [1, 3, 9])
def test_sweep_no_pt(N, n_traj):
    sysd, grid = H.random_system(N, n_steps=30, seed=N)
    tr = _traj(grid.n_steps, N, n_traj, seed=N + n_traj)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, N - 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr), oracle.propagate(sysd, grid, rho0, ops, tr), 1e-12)


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("chi", [8, 16, 32, 64, 100, 128])
def test_sweep_pt(N, chi):
    if chi > 64 and N > 4:
        pytest.skip("chi > 64 is built for N^2 <= 16 (LDS)")
    sysd, grid = H.random_system(N, n_steps=24, seed=3 * N + chi)
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=7, seed=chi, eps=0.15)
    tr = _traj(grid.n_steps, N, 6, seed=N * chi)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt), 1e-11)


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("chi", [16, 32, 64])
@pytest.mark.parametrize("split", ["0", "2g", "2c", "2c-noxcd", "2c-noow"])
def test_sweep_pt_split_groups(monkeypatch, N, chi, split):
    """small batches: each trajectory over N^2 (+ 1) workgroups gathering its state through global memory once per
    step (pt_split.hip), forced (2g: data-tagged granule exchange; 2c: the counter exchange with the output
    workgroup, the default; both with each group's workgroups dealt onto one XCD; 2c-noxcd: the plain grid;
    2c-noow: the counter exchange with workgroup 0 writing the outputs) and off (0), with MTOs of every kind (uneven
    work per group), ragged windows, several systems and a repeated slice (the slice row kept in registers across
    steps); the forced cases check that the plan really ran split groups"""
    monkeypatch.setenv("PQD_SPLIT", split[0])
    monkeypatch.setenv("PQD_SPLIT_GRAN", "1" if split == "2g" else "0")
    monkeypatch.setenv("PQD_SPLIT_XCD", "0" if split.endswith("noxcd") else "1")
    monkeypatch.setenv("PQD_SPLIT_OW", "0" if split.endswith("noow") else "1")
    systems = [H.random_system(N, n_steps=30, seed=40 + k)[0] for k in range(3)]
    grid = Grid(0.0, 0.1, 30)
    n_traj = max(1, min(7, 256 // (N * N + 1)))  # every group resident (N^2 + 1 workgroups with the output one)
    tr = _traj(grid.n_steps, N, n_traj, seed=N + chi)
    tr.system = np.array([k % 3 for k in range(n_traj)])
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=9, seed=chi + N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    if split != "0":
        assert plan.info()[0] == "split groups" and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("N", [3, 4, 6])
@pytest.mark.parametrize("mode", ["l2sc1", "spread"])
def test_sweep_pt_split_groups_exchange_flavours(monkeypatch, N, mode):
    """the counter exchange on the XCD-grouped grid with sc1 stores (PQD_SPLIT_L2=0) instead of the L2-kept lines,
    and a group that reports a spread placement (PQD_ABLATE=512: workgroup 0 claims the next XCD; the first poll sees
    it, the launch ends before its first gather and the plan re-runs the batch on the batched kernel), vs the oracle"""
    monkeypatch.setenv("PQD_SPLIT", "2")
    if mode == "l2sc1":
        monkeypatch.setenv("PQD_SPLIT_L2", "0")
    else:
        monkeypatch.setenv("PQD_ABLATE", "512")
    systems = [H.random_system(N, n_steps=30, seed=50 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 30)
    n_traj = max(1, min(5, 256 // (N * N + 1)))
    tr = _traj(grid.n_steps, N, n_traj, seed=2 * N + 1)
    tr.system = np.array([k % 2 for k in range(n_traj)])
    pt = ptmod.random_pt(N, 64, D=min(N * N, 9), n_slices=6, seed=N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    if mode == "l2sc1" or N * N + 1 > 32:  # (groups of more than 32 workgroups keep one counter and sc1 stores)
        assert plan.info()[0] == "split groups" and plan.info()[2] == 0
    else:
        assert plan.info()[2] == 1 and plan.info()[0] == "batched lock-step sweep"
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("N", [3, 4, 6])
def test_sweep_pt_split_groups_in_consecutive_launches(N):
    """a small batch just above the co-resident capacity (n_traj * N^2 > CUs) runs its split groups as consecutive
    launches (auto mode): same outputs as the oracle and the batched kernel, and the plan reports split groups"""
    chi = 16
    systems = [H.random_system(N, n_steps=30, seed=70 + k)[0] for k in range(2)]
    grid = Grid(0.0, 0.1, 30)
    n_traj = 256 // (N * N) + 2
    tr = _traj(grid.n_steps, N, n_traj, seed=3 * N)
    tr.system = np.array([k % 2 for k in range(n_traj)])
    pt = ptmod.random_pt(N, chi, D=min(N * N, 9), n_slices=9, seed=N, eps=0.15)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0)]
    rho0 = H.random_rho(N)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert plan.info()[0] == "split groups" and plan.info()[2] == 0
    cmp_lists(got, oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


def test_sweep_pt_split_full_c3_single_run(monkeypatch):
    """C3 single run (one biexciton trajectory, chi = 64, 2000 steps): split groups vs the batched kernel"""
    N, chi = 4, 64
    sysd, grid = H.random_system(N, n_steps=2000, seed=7)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=300, seed=11, eps=0.1)
    tr = Trajectories(np.array([0]), np.array([2000]))
    ops = [H.ketbra(N, a, a) for a in range(N)]
    rho0 = H.ketbra(N, 0, 0)
    monkeypatch.setenv("PQD_SPLIT", "2")
    a = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    monkeypatch.setenv("PQD_SPLIT", "0")
    b = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    cmp_lists(a, b, 1e-11)


@pytest.mark.parametrize("fpm", ["0", "1"])
@pytest.mark.parametrize("N,n_sub,dt", [(2, 1, 0.1), (2, 2, 1.0), (2, 3, 2.0), (2, 1, 5.0), (4, 1, 0.1), (4, 2, 1.0),
                                        (4, 1, 2.0), (5, 1, 0.1), (5, 2, 1.0), (6, 1, 0.1), (6, 1, 1.0), (6, 3, 2.0)])
def test_free_propagators_large_n_mfma_and_lds(monkeypatch, fpm, N, n_sub, dt):
    """N2 = 16 / 25 / 36 on the matrix-core kernel (free_prop_mfma_kernel, 4 x 4 blocks, 25 padded to 28) and on
    the LDS kernel (PQD_FPM=0), vs the oracle: norms from ~0.5 to several (dt = 1, 2, 5: squarings), sub-steps (Acc
    products). N2 = 4: the packed kernel's matrix-core products (four matrices per wave, each with its own degree and
    squaring count) and its shuffle products (PQD_FPM=0)"""
    monkeypatch.setenv("PQD_FPM", fpm)
    sysd, grid = H.random_system(N, n_steps=12, n_sub=n_sub, dt=dt, seed=7 * N + n_sub)
    got = engine.free_propagators(sysd, grid)
    ref = oracle.free_propagators(sysd, grid)
    assert rel(got, ref) < 1e-12


@pytest.mark.parametrize("fp4", ["0", "1"])
def test_free_propagators_beyond_32bit_dispatch(monkeypatch, fp4):
    """a scan whose free propagators need more than 2^32 work-items in one-workgroup-per-matrix form
    (1700 systems x 2 x 5000 half steps = 17M matrices x 256 threads): the kernels loop over a capped grid.
    All systems are identical, so every trajectory's last outputs must agree exactly with the first's."""
    monkeypatch.setenv("PQD_FP4", fp4)
    N, n_sys, n_steps = 2, 1700, 5000
    sysd, grid = H.random_system(N, n_chan=1, n_lind=1, seed=5, n_steps=n_steps)
    tr = Trajectories(np.full(n_sys, n_steps - 1), np.full(n_sys, n_steps))
    tr.system = np.arange(n_sys)
    out = engine.propagate([sysd] * n_sys, grid, H.ketbra(N, 0, 0), [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)], tr)
    ref = out[0]
    assert np.all(np.isfinite(ref)) and np.abs(ref).max() > 0
    for k in (1, n_sys // 2, n_sys - 1):
        np.testing.assert_array_equal(out[k], ref)


def test_sweep_pt_many_trajectories_and_ragged_windows():
    N, chi = 4, 64
    sysd, grid = H.random_system(N, n_steps=40, seed=99)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=41, seed=5, eps=0.1)
    tr = _traj(grid.n_steps, N, 37, seed=1)
    ops = [H.ketbra(N, a, b) for a in range(N) for b in range(N)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("chi", [1, 32, 64])
def test_output_tables_match_flat_outputs(chi):
    """pqd_propagate_table / Plan.download_table (ACE's table per trajectory, assembled on the device) hold exactly
    the flat outputs plus the time row (ragged windows, two systems, the no-PT, quad and batched paths)"""
    N = 2 if chi == 32 else 4
    s1, grid = H.random_system(N, n_steps=40, seed=3, ta=-1.25)
    s2, _ = H.random_system(N, n_steps=40, seed=4, ta=-1.25)
    pt = ptmod.random_pt(N, chi, D=N * N, n_slices=41, seed=5, eps=0.1) if chi > 1 else None
    tr = _traj(grid.n_steps, N, 21, seed=2)
    tr = Trajectories(tr.out_begin, tr.out_end, tr.mtos, system=np.arange(tr.n_traj) % 2)
    ops = [H.ketbra(N, a, b) for a in range(N) for b in range(N)][:5]
    rho0 = H.random_rho(N)
    flat = engine.propagate([s1, s2], grid, rho0, ops, tr, pt=pt)
    want = engine.tables_from_outputs(flat, tr, grid)
    got = engine.propagate_table([s1, s2], grid, rho0, ops, tr, pt=pt)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.shape == w.shape and np.array_equal(g, w)
    plan = engine.Plan([s1, s2], grid, rho0, ops, tr, pt=pt)
    plan.execute()
    for g, w in zip(plan.download_table(), want):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("chi", [1, 16, 32])
def test_output_trapz_matches_host_integrals(chi):
    """pqd_propagate_trapz / Plan-free device reduction (the G2_reuse tau integral, pol_entanglement/G2.py:484-505):
    dx (y_head(0) / 2 + interior of y_tail + y_tail(L-1) / 2) per trajectory and pair, vs the same sum over the flat
    outputs on the host; windows of 1 (-> 0), 2 and many steps, ragged, two systems; out-of-range pairs refused"""
    N = 2 if chi == 32 else 4
    s1, grid = H.random_system(N, n_steps=40, seed=3)
    s2, _ = H.random_system(N, n_steps=40, seed=4)
    pt = ptmod.random_pt(N, chi, D=N * N, n_slices=41, seed=5, eps=0.1) if chi > 1 else None
    tr = _traj(grid.n_steps, N, 21, seed=2)
    b, e = tr.out_begin.copy(), tr.out_end.copy()
    b[0], e[0] = 7, 7      # one step: no interval
    b[1], e[1] = 3, 4      # two steps: head and last tail point only
    tr = Trajectories(b, e, tr.mtos, system=np.arange(tr.n_traj) % 2)
    ops = [H.ketbra(N, a, c) for a in range(N) for c in range(N)][:5]
    rho0 = H.random_rho(N)
    no = len(ops)
    kh, kt, dx = [no - 2, no - 1, 0], [0, 1, 2], 0.25
    got = engine.propagate_trapz([s1, s2], grid, rho0, ops, tr, kh, kt, dx, pt=pt)
    flat = engine.propagate([s1, s2], grid, rho0, ops, tr, pt=pt)
    assert got.shape == (tr.n_traj, 3)
    for t, y in enumerate(flat):
        for q in range(3):
            L = y.shape[0]
            want = 0.0 if L < 2 else dx * (0.5 * y[0, kh[q]] + y[1: L - 1, kt[q]].sum() + 0.5 * y[L - 1, kt[q]])
            assert abs(got[t, q] - want) <= 1e-13 * max(1.0, abs(want))
    assert np.all(got[0] == 0)
    with pytest.raises(ValueError, match="not in"):
        engine.propagate_trapz([s1, s2], grid, rho0, ops, tr, [no], [0], dx, pt=pt)


def test_empty_batch_and_zero_steps():
    sysd, grid = H.random_system(2, n_steps=0, seed=0)
    tr = Trajectories(np.array([0]), np.array([0]))
    out = engine.propagate(sysd, grid, H.ketbra(2, 0, 0), [np.eye(2)], tr)
    assert out[0].shape == (1, 1) and abs(out[0][0, 0] - 1) < 1e-15
    out = engine.propagate(sysd, Grid(0, 0.1, 5), H.ketbra(2, 0, 0), [np.eye(2)], Trajectories(np.array([]), np.array([])))
    assert out == []


def test_invalid_arguments_raise():
    sysd, grid = H.random_system(2, n_steps=5, seed=0)
    with pytest.raises(ValueError, match="window"):
        engine.propagate(sysd, grid, H.ketbra(2, 0, 0), [np.eye(2)], Trajectories(np.array([0]), np.array([6])))
    with pytest.raises(ValueError, match="MTO"):
        engine.propagate(sysd, grid, H.ketbra(2, 0, 0), [np.eye(2)],
                         Trajectories(np.array([0]), np.array([5]), [MTO(0, 9, False, 1, np.eye(2))]))
    from pyaceqd_amd import _lib
    with pytest.raises(_lib.PQDError, match="chi 257"):  # (129..256 run on split groups since round 6)
        engine.propagate(sysd, grid, H.ketbra(2, 0, 0), [np.eye(2)], Trajectories(np.array([0]), np.array([5])),
                         pt=ptmod.random_pt(2, 257, n_slices=2))
    s6, g6 = H.random_system(6, n_steps=3, seed=0)
    with pytest.raises(_lib.PQDError, match="CHI=128"):
        engine.propagate(s6, g6, H.ketbra(6, 0, 0), [np.eye(6)], Trajectories(np.array([0]), np.array([3])),
                         pt=ptmod.random_pt(6, 100, D=4, n_slices=2))


# --------------------------------------------------------------------------------- full-size properties (C3)
def test_c3_full_size_invariants():
    """biexciton N=4, chi=64, 10,000 steps: structured PT == bare dynamics; trace preserved"""
    from pyaceqd_amd.four_level_system.linear import biexciton_ops
    from pyaceqd_amd import opgrammar
    from pyaceqd_amd.constants import hbar
    N, dt, n = 4, 0.1, 10000
    so, bo, lo, io, _ = biexciton_ops(delta_b=4, lindblad=True)
    from pyaceqd_amd.pulses import ChirpedPulse, PulseTrain
    train = PulseTrain(100, 10, ChirpedPulse(tau_0=3, e_start=-2.0, e0=1.0, t0=12))
    ds = dt / 4
    ts = ds * np.arange(4 * n + 1)
    fx = train.get_total(ts)
    sysd = System(dim=N, H0=sum(opgrammar.to_matrix(s, N) for s in so),
                  lindblad=[(r, opgrammar.to_matrix(o, N)) for o, r in lo],
                  channels=[(-0.5 * np.pi * hbar * opgrammar.to_matrix(io[0][0], N), fx)], sample_dt=ds)
    grid = Grid(0.0, dt, n)
    pt = ptmod.synthetic_pt(opgrammar.to_matrix(bo, N), chi=64, n_init=410, n_rep=1)
    ops = [opgrammar.to_matrix(f"|{k}><{k}|_4", N) for k in range(4)] + [np.eye(N)]
    tr = Trajectories(np.zeros(8, dtype=int), np.full(8, n))
    rho0 = H.ketbra(N, 0, 0)
    a = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    b = engine.propagate(sysd, grid, rho0, ops, tr)
    for x, y in zip(a, b):
        assert np.max(np.abs(x - y)) < 1e-10
        assert np.max(np.abs(x[:, -1] - 1)) < 1e-10
    # the pulse train actually drives the system
    assert np.max(np.abs(b[0][:, 3])) > 1e-3


# --------------------------------------------------------------------------------- plan API
def test_plan_repeat_is_deterministic():
    N = 4
    sysd, grid = H.random_system(N, n_steps=50, seed=4)
    pt = ptmod.random_pt(N, 32, D=9, n_slices=4, seed=1, eps=0.1)
    tr = _traj(grid.n_steps, N, 10, seed=2)
    ops = [H.ketbra(N, 1, 1)]
    plan = engine.Plan(sysd, grid, H.random_rho(N), ops, tr, pt=pt)
    plan.execute()
    a = plan.download()
    plan.execute(rebuild_free=False)
    plan.execute()
    b = plan.download()
    f, w, k = plan.timing()
    assert k == 3 and w > 0 and f >= 0
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


# --------------------------------------------------------------------------------- map-chain sweeps vs Fortran
def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


@pytest.mark.parametrize("dim", [2, 4, 6])
def test_mapchain_vs_fortran_golden(golden_dir, dim):
    from pyaceqd_amd.two_time import propagate_tau_module as M
    z = load(golden_dir, f"fortran_propagate_tau_d{dim}.npz")
    assert rel(M.propagate_tau(F(z["dm_tl"]), z["rho_init"], int(z["n_tau"]), dim, int(z["j_start"])), z["rho_out"]) < 1e-12
    z = load(golden_dir, f"fortran_onetime_d{dim}.npz")
    r = M.calc_onetime_parallel(F(z["dm_tl"]), z["rho_init"], int(z["n_tau"]), dim, z["opa"], z["opb"], z["opc"],
                                z["time"], z["time_sparse"])
    assert rel(r, z["result"]) < 1e-12
    z = load(golden_dir, f"fortran_onetime_block_d{dim}.npz")
    r = M.calc_onetime_parallel_block(dm_block=F(z["dm_block"]), dm_s=z["dm_s"], rho_init=z["rho_init"],
                                      n_tb=int(z["n_tb"]), nx_tau=int(z["nx_tau"]), dim=dim, opa=z["opa"],
                                      opb=z["opb"], opc=z["opc"], time=z["time"], time_sparse=z["time_sparse"])
    assert rel(r, z["result"]) < 1e-12
    z = load(golden_dir, f"fortran_twotime_phonon_block_d{dim}.npz")
    r = M.calc_twotime_phonon_block(dm_taucs2=np.asfortranarray(z["dm_taucs2"].transpose(2, 3, 0, 1)),
                                    dm_sep1=F(z["dm_sep1"]), dm_sep2=F(z["dm_sep2"]), dm_s=z["dm_s"],
                                    rho_init=z["rho_init"], n_tb=int(z["n_tb"]), nx_tau=int(z["nx_tau"]), dim=dim,
                                    opa=z["opa"], opb=z["opb"], opc=z["opc"], time=z["time"],
                                    time_sparse=z["time_sparse"])
    assert rel(r, z["result"]) < 1e-12


@pytest.mark.parametrize("dim", [2, 4, 5])
def test_timebin_vs_fortran_golden(golden_dir, dim):
    from pyaceqd_amd.timebin import timebin_tl as TB
    z = load(golden_dir, f"fortran_timebin_d{dim}.npz")
    a = (F(z["dm_1"]), F(z["dm_2"]), z["rho_init"], z["t1"], F(z["precalc"]), float(z["dt"]), dim)
    o = list(z["ops8"])
    tb = float(z["tb"])
    assert rel(TB.four_time_8op(*a, *o, False, False, tb), z["result8"]) < 1e-12
    assert rel(TB.four_time_8op(*a, *o, True, False, tb), z["result8_early"]) < 1e-12
    assert rel(TB.four_time_8op(*a, *o, False, True, tb), z["result8_late"]) < 1e-12
    assert rel(TB.four_time(*a, *o[:4], tb), z["result4"]) < 1e-12
    assert rel(TB.dynamics_t1(*a, tb), z["dyn_t1"]) < 1e-12


def test_mapchain_large_vs_oracle():
    """C4-shaped map-chain sweep (256 t1 points x 2000 tau steps, N=4) vs the C oracle"""
    from pyaceqd_amd.two_time import propagate_tau_module as M
    rng = np.random.default_rng(0)
    dim, n_tau = 4, 2000
    N2 = dim * dim
    n_tfull = 256 + n_tau + 2
    base = np.eye(N2) + 0.02 * (rng.normal(size=(N2, N2)) + 1j * rng.normal(size=(N2, N2)))
    base /= np.max(np.abs(np.linalg.eigvals(base)))
    maps = np.stack([base] * (n_tfull - 1)) * (1 + 1e-4 * rng.normal(size=(n_tfull - 1, 1, 1)))
    time = np.round(np.arange(n_tfull) * 0.1, 6)
    ts = np.round(np.arange(256) * 0.1, 6)
    ops = [rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)) for _ in range(3)]
    rho = H.random_rho(dim).reshape(N2)
    a = M.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts)
    b = oracle.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts, nthreads=8)
    assert rel(a, b) < 1e-11


@pytest.mark.parametrize("dim", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("L", ["8", "13", "0"])
def test_mapchain_blocked_sweep_vs_oracle(monkeypatch, dim, L):
    """calc_onetime_parallel on the blocked sweep (per-block prefix products, mapchain.hip mcb_*) for block lengths
    8 / 13 / auto (sqrt(n_tau)), trajectories that start on, just before and just after block boundaries, repeated
    and off-grid t1 points, a t1 point past the grid, vs the C oracle and vs the map-by-map pipelined kernel"""
    from pyaceqd_amd.two_time import propagate_tau_module as M
    if L != "0":
        monkeypatch.setenv("PQD_MC_L", L)
    rng = np.random.default_rng(dim)
    N2 = dim * dim
    n_tau, n_tfull = 150, 260
    maps = np.stack([np.eye(N2) + 0.05 * (rng.normal(size=(N2, N2)) + 1j * rng.normal(size=(N2, N2))) / dim
                     for _ in range(n_tfull - 1)])
    time = np.round(np.arange(n_tfull) * 0.1, 6)
    ts = np.array([0.0, 0.05, 0.7, 0.75, 0.8, 0.8, 1.2, 1.3, 1.31, 2.55, 4.0, 6.4, 7.9, 10.0, 10.85])
    ops = [rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)) for _ in range(3)]
    rho = H.random_rho(dim).reshape(N2)
    a = M.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts)
    b = oracle.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts, nthreads=8)
    assert rel(a, b) < 1e-11
    monkeypatch.setenv("PQD_MC_BLOCKED", "0")
    c = M.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts)
    assert rel(a, c) < 1e-11


@pytest.mark.parametrize("dim", [2, 4, 6])
@pytest.mark.parametrize("L", ["8", "0"])
@pytest.mark.parametrize("n_map", [7, 18])
def test_mapchain_blocked_sweep_block_mode_vs_oracle(monkeypatch, dim, L, n_map):
    """calc_onetime_parallel_block on the blocked sweep: the periodic map sequence (dm_block for the first n_map of
    every n_tb, then dm_s), trunks ending inside and past the first period (those apply dm_s at every tau step,
    propagate_tau.f90:270-287), vs the C oracle and the map-by-map kernel. n_map = 18 > n_tb = 12 puts trunk ends
    inside (n_tb, n_map] (t1 = 1.2, 1.25: they walk dm_block(j..n_map) before dm_s), which the host routes to the
    map-by-map kernels"""
    from pyaceqd_amd.two_time import propagate_tau_module as M
    if L != "0":
        monkeypatch.setenv("PQD_MC_L", L)
    rng = np.random.default_rng(10 + dim)
    N2 = dim * dim
    n_tb, nx_tau = 12, 9
    mk = lambda: np.eye(N2) + 0.05 * (rng.normal(size=(N2, N2)) + 1j * rng.normal(size=(N2, N2))) / dim  # noqa
    dm_block = np.stack([mk() for _ in range(n_map)])
    dm_s = mk()
    time = np.round(np.arange(60) * 0.1, 6)
    ts = np.array([0.0, 0.15, 0.4, 0.75, 1.1, 1.2, 1.25, 2.0, 3.3])
    ops = [rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)) for _ in range(3)]
    rho = H.random_rho(dim).reshape(N2)
    args = (F(dm_block), np.asfortranarray(dm_s), rho, n_tb, nx_tau, dim, *ops, time, ts)
    a = M.calc_onetime_parallel_block(*args)
    b = oracle.calc_onetime_parallel_block(*args)
    assert rel(a, b) < 1e-11
    monkeypatch.setenv("PQD_MC_BLOCKED", "0")
    c = M.calc_onetime_parallel_block(*args)
    assert rel(a, c) < 1e-11


@pytest.mark.parametrize("dim", [2, 3, 4, 5, 6])
def test_map_tail_vs_oracle(dim):
    """pqd_map_tail (the tau tails of the phonon dynamical-map correlations, correlations.py:866-1186) vs the
    reference loop restated in oracle.map_tail: 37 rows (ragged against the rows packed per wave), 1,500 steps"""
    from pyaceqd_amd.two_time import propagate_tau_module as M
    rng = np.random.default_rng(70 + dim)
    N2 = dim * dim
    Mm = np.eye(N2) + 0.05 * (rng.normal(size=(N2, N2)) + 1j * rng.normal(size=(N2, N2))) / dim
    X = rng.normal(size=(N2, 37)) + 1j * rng.normal(size=(N2, 37))
    w = rng.normal(size=N2) + 1j * rng.normal(size=N2)
    a = M.map_tail(Mm, X, w, 1500)
    b = oracle.map_tail(Mm, X, w, 1500)
    assert a.shape == (37, 1500)
    assert rel(a, b) < 1e-12


def test_mapchain_blocked_refuses_reads_past_the_maps():
    """a tau window running past the last map is refused (the Fortran would read past dm_tl)"""
    from pyaceqd_amd.two_time import propagate_tau_module as M
    dim, N2, n_tfull = 2, 4, 30
    maps = np.stack([np.eye(N2, dtype=complex)] * (n_tfull - 1))
    time = np.round(np.arange(n_tfull) * 0.1, 6)
    ops = [np.eye(dim, dtype=complex)] * 3
    with pytest.raises(ValueError, match="would read map"):
        M.calc_onetime_parallel(F(maps), np.eye(dim, dtype=complex).reshape(N2), 25, dim, *ops, time,
                                np.array([0.0, 0.5]))


# --------------------------------------------------------------------------------- time-local maps
def test_tl_dynmap_vs_reference_golden(golden_dir):
    """GPU Jacobi-SVD pinv time-localisation vs the reference's calc_tl_dynmap_pseudo (tools.py:446-484)
    at map sizes 4/16/25/36, including rank-deficient maps where the rcond=1e-12 cut-off drops 3 singular
    values (tests/golden/make_golden_tlmap.py, pyref_tools.npz)"""
    from pyaceqd_amd import tools as T
    z = load(golden_dir, "pyref_tlmap.npz")
    for name in ("d4", "d5", "d6", "rank2", "rank4"):
        got = T.calc_tl_dynmap_pseudo(z[f"{name}_dm"], z[f"{name}_times"])
        assert got.shape == z[f"{name}_tl"].shape
        assert rel(got, z[f"{name}_tl"]) < 1e-10, name
    z = load(golden_dir, "pyref_tools.npz")
    assert rel(T.calc_tl_dynmap_pseudo(z["dm_cum"], z["tl_times"]), z["tl_maps"]) < 1e-10
    # fewer maps than times-1 is an error, as the reference's indexing would be
    with pytest.raises(ValueError):
        T.calc_tl_dynmap_pseudo(z["dm_cum"][:3], z["tl_times"])


@pytest.mark.parametrize("dim,n_maps", [(2, 3000), (4, 3000), (6, 400)])
def test_tl_dynmap_large_vs_oracle(dim, n_maps):
    """long map chains: GPU vs the numpy-pinv oracle, and the size-independent property that
    time-localising the cumulative products of per-step maps gives back those maps"""
    from pyaceqd_amd import tools as T
    rng = np.random.default_rng(dim)
    N2 = dim * dim
    G = 0.05 * (rng.normal(size=(N2, N2)) + 1j * rng.normal(size=(N2, N2)))
    steps = np.empty((n_maps, N2, N2), dtype=complex)
    import scipy.linalg as sla
    base = sla.expm(G - G.conj().T)  # unitary: the cumulative maps stay well conditioned
    for i in range(n_maps):
        steps[i] = base @ (np.eye(N2) + 1e-3 * np.sin(0.01 * i) * (G + G.conj().T))
    dm = np.empty_like(steps)
    acc = np.eye(N2, dtype=complex)
    for i in range(n_maps):
        acc = steps[i] @ acc
        dm[i] = acc
    times = np.round(np.arange(n_maps + 1) * 0.1, 6)
    got = T.calc_tl_dynmap_pseudo(dm, times)
    assert rel(got, oracle.tl_dynmap_pseudo(dm)) < 1e-9
    assert rel(got, steps) < 1e-9


# --------------------------------------------------------------------------------- drop-in driver
def _oracle_patch(monkeypatch):
    """route general_system's propagate through the oracle (same lowering, CPU arithmetic)"""
    from pyaceqd_amd.general_system import general_system as gs

    def prop(system, grid, rho0, out_ops, traj, pt=None, ctx=None):
        return oracle.propagate(system, grid, rho0, out_ops, traj, pt=pt, nthreads=8)
    monkeypatch.setattr(gs, "propagate", prop)
    monkeypatch.setattr(gs, "propagate_table", lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None:
                        engine.tables_from_outputs(prop(system, grid, rho0, out_ops, traj, pt), traj, grid))


@pytest.mark.parametrize("sampling", ["ace_file", "exact"])
def test_tls_rabi_kat(sampling):
    """area theorem: a resonant pulse of area pi e0 leaves sin^2(pi e0 / 2) in |1>. With the default ("ace_file",
    the reference's %.8f files on np.arange(t_start, t_end, dt), linearly interpolated) the two half-step midpoints of
    a step weigh the samples like the trapezoid rule, so the area is exact to the %.8f quantisation"""
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.pulses import ChirpedPulse
    for e0 in (0.5, 1.0, 2.0):
        t, g, x, p, _ = tls(0, 40, ChirpedPulse(tau_0=3, e_start=0, e0=e0, t0=20), dt=0.05, pulse_sampling=sampling)
        assert abs(x[-1].real - np.sin(np.pi * e0 / 2) ** 2) < 1e-6
        assert np.max(np.abs(g + x - 1)) < 1e-12


def test_tls_c1_vs_oracle(monkeypatch):
    """config C1: tls(0,100, ChirpedPulse(tau_0=3, e_start=0, e0=1, t0=20), dt=0.1, lindblad=True)"""
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.pulses import ChirpedPulse
    args = dict(dt=0.1, lindblad=True)
    p = ChirpedPulse(tau_0=3, e_start=0, e0=1, t0=20)
    a = tls(0, 100, p, **args)
    assert a.shape == (5, 1001)
    _oracle_patch(monkeypatch)
    b = tls(0, 100, p, **args)
    assert np.max(np.abs(a - b)) < 1e-12


def test_biexciton_and_sixls_vs_oracle(monkeypatch, tmp_path):
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.six_level_system.linear import sixls_linear
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd import opgrammar
    pfile = str(tmp_path / "bx.npz")
    ptmod.save_pt(pfile, ptmod.random_pt(4, 32, D=9, n_slices=30, seed=3, eps=0.05), dim=4)
    p = ChirpedPulse(tau_0=3, e_start=-2.0, e0=1.0, t0=12, polar_x=0.8)
    runs = [lambda: biexciton(0, 30, p, dt=0.1, delta_xy=0.02, lindblad=True, phonons=True, pt_file=pfile),
            lambda: sixls_linear(0, 30, p, dt=0.1, bx=2.0, bz=0.5, lindblad=True, output_dm=True)]
    got = [r() for r in runs]
    _oracle_patch(monkeypatch)
    ref = [r() for r in runs]
    assert rel(got[0], ref[0]) < 1e-11
    assert rel(got[1][1], ref[1][1]) < 1e-12


def test_three_op_two_time_vs_oracle(monkeypatch, tmp_path):
    """C4-shaped two-time G2 sweep through the batched driver (small sizes)"""
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.two_time.correlations import three_op_two_time
    from pyaceqd_amd.pulses import ChirpedPulse
    pfile = str(tmp_path / "bx.npz")
    ptmod.save_pt(pfile, ptmod.synthetic_pt(np.diag([0, 1, 1, 2.0]), chi=16, n_init=20, n_rep=2, structured=False,
                                             eps=0.05), dim=4)
    p = ChirpedPulse(tau_0=3, e_start=-2.0, e0=1.0, t0=5)
    t_axis = np.round(np.arange(12) * 0.5, 6)
    kw = dict(opA="|3><1|_4", opB="|1><1|_4", opC="|1><3|_4", tau_max=8.0, dt=0.1)
    opts = lambda: {"lindblad": True, "phonons": True, "pt_file": pfile}  # noqa: E731
    t1, tau, G = three_op_two_time(biexciton, t_axis, p, options=opts(), **kw)
    assert G.shape == (12, 81)
    _oracle_patch(monkeypatch)
    _, _, Gr = three_op_two_time(biexciton, t_axis, p, options=opts(), **kw)
    assert rel(G, Gr) < 1e-10


def test_calc_dynmap_consistency():
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.pulses import ChirpedPulse
    p = ChirpedPulse(tau_0=2, e_start=0.1, e0=1.3, t0=5)
    rho0 = np.array([[0.7, 0.2], [0.2, 0.3]], dtype=complex)
    res, dm = tls(0, 10, p, dt=0.1, lindblad=True, calc_dynmap=True, rho0=rho0)
    direct = tls(0, 10, p, dt=0.1, lindblad=True, rho0=rho0)
    assert dm.shape == (100, 4, 4)
    assert np.max(np.abs(res - direct)) < 1e-12
    rho_end = (dm[-1] @ rho0.reshape(4)).reshape(2, 2)
    assert abs(rho_end[1, 1] - direct[2][-1]) < 1e-12


# --------------------------------------------------------------------------------- B = 8 workgroups, scans
@pytest.mark.parametrize("N", [2, 3, 4])
@pytest.mark.parametrize("chi", [16, 32, 64])
def test_sweep_pt_bt8(monkeypatch, N, chi):
    monkeypatch.setenv("PQD_BT", "8")
    sysd, grid = H.random_system(N, n_steps=20, seed=5 * N + chi)
    pt = ptmod.random_pt(N, chi, D=min(N * N, 7), n_slices=9, seed=chi + 1, eps=0.15)
    tr = _traj(grid.n_steps, N, 19, seed=N + chi)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("bt", ["4", "8"])
@pytest.mark.parametrize("with_pt", [False, True])
def test_multi_system_scan(monkeypatch, with_pt, bt, fuse):
    """trajectories of several systems; workgroups straddle systems (each wave reads its own system's free
    propagators and fused output maps; the lane-parallel traces prefetch each trajectory's own W rows)"""
    monkeypatch.setenv("PQD_BT", bt)
    monkeypatch.setenv("PQD_FUSE", fuse)
    N = 4
    systems = [H.random_system(N, n_steps=30, seed=20 + k)[0] for k in range(5)]
    grid = Grid(0.0, 0.1, 30)
    tr = _traj(grid.n_steps, N, 21, seed=9)
    tr.system = np.array([k % 5 for k in range(21)])
    pt = ptmod.random_pt(N, 32, D=9, n_slices=5, seed=3, eps=0.1) if with_pt else None
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 3, 0)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(systems, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("trpre", ["0", "1"])
@pytest.mark.parametrize("fuse", ["0", "1"])
def test_bench_workload_small_vs_oracle(monkeypatch, fuse, trpre):
    """the bench workload itself (scan of G2 sweeps, chi=64, B=8 path) at reduced n_tau vs the oracle,
    with the fused half steps (default) and without"""
    monkeypatch.setenv("PQD_FUSE", fuse)
    monkeypatch.setenv("PQD_TRPRE", trpre)
    import bench
    systems, grid, pt, rho0, ops, tr = bench.build_workload(16, 60, 64, scan=2)
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    ref = oracle.propagate(systems, grid, rho0, ops, tr, pt=pt, nthreads=8)
    cmp_lists(got, ref, 1e-11)


@pytest.mark.parametrize("pt_mode", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("bt", [4, 8])
@pytest.mark.parametrize("N,chi", [(2, 16), (3, 32), (4, 64), (5, 64), (6, 32), (2, 128), (4, 128)])
@pytest.mark.parametrize("fuse", ["0", "1"])
def test_sweep_pt_contraction_modes(monkeypatch, pt_mode, bt, N, chi, fuse):
    """PT contraction on the VALU (0), on the matrix cores (1, v_mfma_f64_4x4x4_4b; 4, the same with three real
    products per complex product; 3, split-complex v_mfma_f64_16x16x4 at B = 8) and mixed per wave (2); column
    phases alternate between the 4M and 3M complex products"""
    monkeypatch.setenv("PQD_CMUL3", str((pt_mode + bt + chi) % 2))
    if bt == 8 and N > 4:
        pytest.skip("B=8 workgroups are built for N^2 <= 16")
    if bt == 8 and chi > 64:
        pytest.skip("chi = 128 runs B=4 workgroups (LDS)")
    monkeypatch.setenv("PQD_BT", str(bt))
    monkeypatch.setenv("PQD_PT_MODE", str(pt_mode))
    monkeypatch.setenv("PQD_FUSE", fuse)
    sysd, grid = H.random_system(N, n_steps=18, seed=7 * N + chi)
    pt = ptmod.random_pt(N, chi, D=min(N * N, 8), n_slices=6, seed=chi + N, eps=0.15)
    tr = _traj(grid.n_steps, N, 21, seed=2 * N + chi)
    ops = [H.ketbra(N, 0, 0), H.ketbra(N, N - 1, 0), np.eye(N)]
    rho0 = H.random_rho(N)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


@pytest.mark.parametrize("cfg", ["c1", "c2", "c3one", "c5", "c5d", "c3d"])
def test_config_workloads_small_vs_oracle(cfg):
    """the SURVEY §8d configurations measured by scripts/bench_configs.py, at reduced scan size
    and step count, vs the oracle: one system per trajectory (c1, c2), a single trajectory (c3one), the six-level
    G2 scan at N^2 = 36 with and without a dictionary PT (c5, c5d: units of up to 4 rows per slice), the
    biexciton scan with a dictionary PT (c3d)"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import bench_configs
    c = dict(bench_configs.CONFIGS[cfg])
    c["n_scan"] = min(c["n_scan"], 5)
    c["n_t1"] = min(c["n_t1"], 7)
    c["n_tau"] = 40
    N, sysd, grid, pt, rho0, ops, tr = bench_configs.workload(**c)
    cmp_lists(engine.propagate(sysd, grid, rho0, ops, tr, pt=pt),
              oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-11)


# --------------------------------------------------------------------------------- generated phonon PTs
def test_tls_phonons_generated_pt_vs_oracle(monkeypatch, tmp_path):
    """config C2 shape: tls with a generated QD-phonon PT (pyaceqd_amd.ptgen, bond capped at 32 by the threshold
    choice / cap), driver path on the GPU vs the same lowering on the CPU oracle; phonons visibly damp the Rabi
    rotation relative to the phonon-free run"""
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd import ptgen, opgrammar
    eta, delta = ptgen.eta_coefficients(lambda w: ptgen.qd_phonon_J(w, ae=3.0), 4.0, 0.1, 30)
    pt = ptgen.build_gaussian_pt(opgrammar.to_matrix("1.000*|1><1|_2", 2), 0.1, eta, delta, threshold=1e-8,
                                 max_bond=32)
    assert pt.chi == 32
    p = ChirpedPulse(tau_0=3, e_start=0, e0=5, t0=15)
    kw = dict(dt=0.1, lindblad=True, phonons=True, pt_file=pt, temp_dir=str(tmp_path) + "/")
    a = tls(0, 60, p, **kw)
    free = tls(0, 60, p, dt=0.1, lindblad=True)
    _oracle_patch(monkeypatch)
    b = tls(0, 60, p, **kw)
    assert rel(a, b) < 1e-11
    assert np.max(np.abs(a[2] - free[2])) > 1e-2
    # trace: exact without phonons; with the chi=32-capped PT it drifts at the truncation level (~1e-5)
    assert np.max(np.abs(a[1] + a[2] - 1)) < 1e-4


def test_biexciton_generated_pt_two_time_vs_oracle(monkeypatch, tmp_path):
    """biexciton with a generated chi=64 phonon PT (explicit + repeated slices) through the batched G2 sweep"""
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.two_time.correlations import three_op_two_time
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd import ptgen, opgrammar
    eta, delta = ptgen.eta_coefficients(lambda w: ptgen.qd_phonon_J(w, ae=3.0), 4.0, 0.1, 6)
    pt = ptgen.build_gaussian_pt(opgrammar.to_matrix("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4", 4), 0.1, eta, delta,
                                 threshold=1e-10, max_bond=64)
    assert pt.chi == 64 and pt.D == 9
    p = ChirpedPulse(tau_0=3, e_start=-2.0, e0=1.0, t0=5)
    t_axis = np.round(np.arange(8) * 0.5, 6)
    kw = dict(opA="|3><1|_4", opB="|1><1|_4", opC="|1><3|_4", tau_max=6.0, dt=0.1)
    opts = lambda: {"lindblad": True, "phonons": True, "pt_file": pt}  # noqa: E731
    _, _, G = three_op_two_time(biexciton, t_axis, p, options=opts(), **kw)
    _oracle_patch(monkeypatch)
    _, _, Gr = three_op_two_time(biexciton, t_axis, p, options=opts(), **kw)
    assert rel(G, Gr) < 1e-10


# --------------------------------------------------------------------------------- pol-entanglement tomography
def test_pol_entanglement_biexciton_vs_oracle(monkeypatch, tmp_path):
    """PolarizatzionEntanglement on the biexciton cascade (two-photon excitation, fine-structure splitting) through
    the batched driver: GPU vs the oracle for the 10-component density matrix and the time-resolved concurrence;
    the physics gives a strongly entangled, fine-structure-degraded state (0 < C < 1)"""
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.pol_entanglement.G2 import PolarizatzionEntanglement
    from pyaceqd_amd.pulses import ChirpedPulse
    p = ChirpedPulse(tau_0=2.0, e_start=-2.0, e0=np.sqrt(2) * 1.0, t0=8)   # TPE at delta_b = 4 meV

    def run():
        opts = {"gamma_e": 1 / 50, "lindblad": True, "delta_xy": 0.005, "temp_dir": str(tmp_path) + "/"}
        pe = PolarizatzionEntanglement(biexciton, "|0><1|_4+|1><3|_4", "|0><2|_4+|2><3|_4",
                                       "|1><0|_4+|3><1|_4", "|2><0|_4+|3><2|_4", p, dt=0.1, tend=40,
                                       regular_grid=True, dt_small=0.5, options=opts)
        c, rho = pe.calc_densitymatrix_reuse(return_rho=True)
        t1, t2, F = pe.calc_timedep_data()
        t, c_t = pe.calc_timedependent_rho(t1=t1, t2=t2, G2_full=F, mode="t", skip=40)[:2]   # photons exist only after the pulse
        return c, rho, F, c_t
    c, rho, F, c_t = run()
    _oracle_patch(monkeypatch)
    cr, rhor, Fr, c_tr = run()
    assert rel(rho, rhor) < 1e-10 and rel(F, Fr) < 1e-10
    assert abs(c - cr) < 1e-9 and np.max(np.abs(c_t - c_tr)) < 1e-8
    assert 0.3 < c < 1.0


# --------------------------------------------------------------------------------- purity / indistinguishability
def test_indistinguishability_map_sweeps_vs_reference_golden(golden_dir, tmp_path):
    """Indistinguishability(dm=True) G1_tl / G2_tl (calc_onetime_parallel_block) and the phonon variants
    (calc_twotime_phonon_block) on the GPU map-chain kernels vs the reference classes running the reference Fortran
    on the same synthetic maps (tests/golden/pyref_purity.npz, tests/golden/make_golden.py gen_purity)"""
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.two_time.purity import Indistinguishability
    from tests.fake_system import fake_system_dm
    z = np.load(os.path.join(golden_dir, "pyref_purity.npz"))
    p = ChirpedPulse(tau_0=1.5, e_start=0, e0=1, t0=6)
    kw = dict(dt=0.1, tb=20, dt_small=0.5, gaussian_t=12)
    opts = {"gamma_e": 0.01, "temp_dir": str(tmp_path) + "/", "phonons": False}
    tl = Indistinguishability(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options=opts, dm=True, **kw)
    assert rel(tl.G1_tl()[1], z["tl_g1"]) < 1e-11
    assert rel(tl.G2_tl()[1], z["tl_g2"]) < 1e-11
    assert np.max(np.abs(np.array(tl.calc_indistinguishability()) - z["tl_indist"])) < 1e-10
    opts["phonons"] = True
    ph = Indistinguishability(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options=opts, dm=True, t_mem=2, **kw)
    assert rel(ph.G1_tl_phonons()[1], z["ph_g1"]) < 1e-11
    assert rel(ph.G2_tl_phonons()[1], z["ph_g2"]) < 1e-11


def test_purity_tls_driver_vs_oracle(monkeypatch, tmp_path):
    """Purity on the real TLS driver (pulse train, batched G2 trajectories): GPU vs oracle; a resonant pi pulse
    much shorter than the lifetime gives a high single-photon purity (re-excitation keeps it below 1)"""
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.two_time.purity import Purity

    def run():
        pu = Purity(tls, "|0><1|_2", "|1><0|_2", ChirpedPulse(tau_0=1.0, e_start=0, e0=1, t0=5), dt=0.1, tb=60,
                    dt_small=0.5, gaussian_t=10, options={"gamma_e": 1 / 10, "lindblad": True,
                                                          "temp_dir": str(tmp_path) + "/"})
        t2, g2 = pu.G2()
        return g2, pu.calc_purity()
    g2, P = run()
    _oracle_patch(monkeypatch)
    g2r, Pr = run()
    assert rel(g2, g2r) < 1e-10 and abs(P - Pr) < 1e-10
    assert 0.8 < P < 1.0


def test_g1_twols_and_mollow_vs_oracle(monkeypatch, tmp_path):
    """G1_twols (batched t grid) and a two-area pulsed Mollow spectrum on the TLS driver: GPU vs oracle"""
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.two_time import G1 as g1mod
    td = str(tmp_path) + "/"

    def run():
        t, tau, g = g1mod.G1_twols(0, 20, 0, 10, 0.5, 0.1, ChirpedPulse(tau_0=1.0, e_start=0, e0=3, t0=5),
                                   gamma_e=1 / 20, temp_dir=td)
        # the pulsed-Mollow drivers call G1_twols with coarse_t=True, which (reference G1.py:44-48) hands the first
        # pulse to construct_t's dt_exp slot and fails for a single pulse; the spectrum step is exercised directly
        s = g1mod._t_integrated_spectrum(t, tau, g)
        return g, s
    g, s = run()
    _oracle_patch(monkeypatch)
    gr, sr = run()
    assert rel(g, gr) < 1e-10 and rel(s, sr) < 1e-10
    assert abs(g[0, 0]) < 1e-12                      # nothing excited before the pulse


# --------------------------------------------------------------------------------- scans (multi-system launches)
def test_rabi_rotation_scan_one_launch(monkeypatch, tmp_path):
    """RabiRotations: the whole area scan is one multi-system launch; final populations follow sin^2(pi A / 2)
    (resonant, no decay), the emitted-photon scan matches the oracle"""
    from pyaceqd_amd.two_level_system.rabi_rotations import RabiRotations
    rr = RabiRotations(dt=0.05, tau=2, area_max=3, n_area=7, temp_dir=str(tmp_path) + "/")
    areas, x = rr.get_rabi_rotations(integrate=False, path=str(tmp_path / "a_"), delete_pt=False)
    # the pulse is cut at t0 - 4 tau = 0 and 8 tau: the missing Gaussian tails cost ~1e-4 of the area
    assert np.max(np.abs(x - np.sin(np.pi * areas / 2) ** 2)) < 1e-3
    rr2 = RabiRotations(dt=0.1, tau=2, area_max=3, n_area=5, gamma_e=1 / 50, temp_dir=str(tmp_path) + "/")
    _, n_ph = rr2.get_rabi_rotations(integrate=True, path=str(tmp_path / "b_"), delete_pt=False)
    _oracle_patch(monkeypatch)
    rr3 = RabiRotations(dt=0.1, tau=2, area_max=3, n_area=5, gamma_e=1 / 50, temp_dir=str(tmp_path) + "/")
    _, n_ref = rr3.get_rabi_rotations(integrate=True, path=str(tmp_path / "c_"), delete_pt=False)
    assert np.max(np.abs(n_ph - n_ref)) < 1e-10
    assert os.path.isfile(str(tmp_path / "b_rabi_.csv"))


def test_tpe_rotation_scan_vs_oracle(monkeypatch, tmp_path):
    from pyaceqd_amd.four_level_system.tpe_rotations import TPERotations

    def run(tag):
        tp = TPERotations(dt=0.1, tau=3, area_max=4, n_area=5, gamma_e=1 / 50, delta_b=4)
        return tp.get_rabi_rotations(detuning=-2.0, integrate=False, path=str(tmp_path / tag), delete_pt=False)[1]
    a = run("g_")
    _oracle_patch(monkeypatch)
    b = run("o_")
    assert rel(a, b) < 1e-10
    assert a[2].max() > 0.5            # two-photon resonant excitation reaches the biexciton


# --------------------------------------------------------------------------------- time-bin two-photon states
def test_twophoton_timebin_tl_paths_vs_reference_golden(golden_dir, tmp_path):
    """TwoPhotonTimebinNew time-local-map paths (four_time_8op / four_time kernels, utils.fast_propagate) vs the
    reference class with the reference Fortran on the same synthetic maps (tests/golden/pyref_twophoton.npz).
    The time-local maps come from the GPU Jacobi-SVD pinv (tools.calc_tl_dynmap_pseudo), the golden from LAPACK's
    SVD inside numpy's pinv. These damped cumulative maps reach cond = 3.8e10; against a 40-digit inverse both
    pinvs are off by ~3e-7 at the map level (LAPACK 2.7e-7, Jacobi 3.7e-7), and the two differ from each other by
    5e-9 relative in the outputs below. Hence the north-star no-phonon bar, 1e-8, instead of the sweeps' 1e-11."""
    tol = 1e-8
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.timebin.twophoton_new import TwoPhotonTimebinNew
    from tests.fake_system import fake_system_dm
    z = np.load(os.path.join(golden_dir, "pyref_twophoton.npz"))
    ps = [ChirpedPulse(tau_0=1.0, e_start=0, e0=1, t0=3), ChirpedPulse(tau_0=1.0, e_start=0, e0=1, t0=15)]
    opts = {"gamma_e": 0.05, "temp_dir": str(tmp_path) + "/", "fake_dim": 4}
    tl = TwoPhotonTimebinNew(fake_system_dm, "|0><1|_4", "|1><0|_4", "|1><3|_4", "|3><1|_4", *ps, options=opts,
                             dt=0.1, dim=4, tb=12, dt_small=0.5, n_tbig=2, gaussian_t=6)
    c, rho, _ = tl.calc_densitymatrix_tl(reduced=False)
    assert rel(rho, z["tl_rho"]) < tol
    assert rel(tl.eell_tl_f()[3], z["tl_eell_f"]) < tol
    t, r = tl.dynamics_tl()
    assert rel(r, z["tl_dyn_rho"]) < tol
    t, r = tl.dynamics_tl_t1()
    assert rel(r, z["tl_dyn1_rho"]) < tol
    ft = tl.four_time_tl(tl.sigma_bdag, tl.sigma_xdag, tl.sigma_b, tl.sigma_x)
    assert rel(ft[3], z["tl_ft_table"]) < tol


def test_twophoton_timebin_biexciton_vs_oracle(monkeypatch, tmp_path):
    """time-bin entangled pair from the biexciton cascade (two TPE pulses one bin apart): the full direct density
    matrix, whose pair sweeps run as single launches of n(n+1)/2 trajectories, GPU vs oracle"""
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.timebin.twophoton_new import TwoPhotonTimebinNew
    ps = [ChirpedPulse(tau_0=1.5, e_start=-2.0, e0=0.5, t0=6), ChirpedPulse(tau_0=1.5, e_start=-2.0, e0=0.5, t0=36)]

    def run():
        opts = {"gamma_e": 1 / 8, "lindblad": True, "temp_dir": str(tmp_path) + "/"}
        tp = TwoPhotonTimebinNew(biexciton, "|0><1|_4", "|1><0|_4", "|1><3|_4", "|3><1|_4", *ps, options=opts,
                                 dt=0.1, dim=4, tb=30, dt_small=1.0, n_tbig=3, gaussian_t=12)
        return tp.calc_densitymatrix(reduced=False)
    c, rho = run()
    _oracle_patch(monkeypatch)
    cr, rhor = run()
    assert rel(rho, rhor) < 1e-10 and abs(c - cr) < 1e-9
