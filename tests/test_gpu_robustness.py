"""Failure detection and launch-path robustness of libpqd (SURVEY.md §5 "failure detection"). GPU only.

* NaN/Inf outputs raise PQD_ERR_NUMERIC (_lib.NumericError) on every path (no PT, batched PT sweep, split groups);
* a split-group launch whose peers do not all arrive is re-run on the batched kernel (forced here with a zero spin
  budget), gives the oracle's result, and the plan reports the fallback and stays batched;
* the no-PT kernel writes every output when there are more output operators than lanes of a wave;
* the general free-propagator kernel's capped-grid loop (more than 2^32 work-items) at N > 2;
* environment switches read at plan creation take effect within one process (PQD_FP4).
"""
import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import _lib, engine, pt as ptmod
from pyaceqd_amd.engine import MTO, Grid, Trajectories
from tests import helpers as H

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def _bad_system(N, n_steps):
    sysd, grid = H.random_system(N, n_steps=n_steps, seed=3)
    H0 = np.array(sysd.H0, dtype=complex)
    H0[0, 0] = np.nan
    sysd.H0 = H0
    return sysd, grid


@pytest.mark.parametrize("path", ["nopt", "batched", "split"])
def test_nan_outputs_raise_numeric_error(monkeypatch, path):
    N = 4
    sysd, grid = _bad_system(N, 12)
    tr = Trajectories(np.array([0]), np.array([12]))
    pt = None
    if path != "nopt":
        monkeypatch.setenv("PQD_SPLIT", "2" if path == "split" else "0")
        pt = ptmod.random_pt(N, 16, D=9, n_slices=5, seed=1, eps=0.1)
    with pytest.raises(_lib.NumericError):
        engine.propagate(sysd, grid, H.ketbra(N, 0, 0), [H.ketbra(N, 1, 1)], tr, pt=pt)


def test_split_timeout_falls_back_to_batched(monkeypatch):
    N, chi = 4, 32
    sysd, grid = H.random_system(N, n_steps=40, seed=8)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=9, seed=4, eps=0.1)
    A = H.ketbra(N, 1, 0) + 0.3 * np.eye(N)
    tr = Trajectories(np.array([0, 3]), np.array([40, 33]), [MTO(0, 7, False, 1, A), MTO(1, 9, True, 2, A)])
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)]
    rho0 = H.random_rho(N)
    monkeypatch.setenv("PQD_SPLIT", "2")
    monkeypatch.setenv("PQD_SPLIT_SPIN", "0")   # every wait for a peer that has not arrived yet times out
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    assert plan.info()[0] == "split groups"
    plan.execute()
    got = plan.download()
    path, bt, fallbacks = plan.info()
    assert fallbacks == 1 and path == "batched lock-step sweep"
    ref = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-11
    plan.execute()                               # stays on the batched kernel: no second fallback
    plan.synchronize()
    assert plan.info()[2] == 1


def test_split_path_reported(monkeypatch):
    N, chi = 4, 64
    sysd, grid = H.random_system(N, n_steps=10, seed=9)
    pt = ptmod.random_pt(N, chi, D=16, n_slices=4, seed=2, eps=0.1)
    tr = Trajectories(np.array([0]), np.array([10]))
    monkeypatch.setenv("PQD_SPLIT", "1")
    plan = engine.Plan(sysd, grid, H.ketbra(N, 0, 0), [H.ketbra(N, 1, 1)], tr, pt=pt)
    assert plan.info() == ("split groups", 4, 0)
    monkeypatch.setenv("PQD_SPLIT", "0")
    plan = engine.Plan(sysd, grid, H.ketbra(N, 0, 0), [H.ketbra(N, 1, 1)], tr, pt=pt)
    assert plan.info()[0] == "batched lock-step sweep"


@pytest.mark.parametrize("N", [2, 4, 6])
def test_no_pt_more_outputs_than_lanes(N):
    sysd, grid = H.random_system(N, n_steps=20, seed=N)
    rng = np.random.default_rng(N)
    ops = [rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N)) for _ in range(100)]
    tr = Trajectories(np.array([0, 5, 2]), np.array([20, 17, 20]), [MTO(1, 6, False, 1, H.ketbra(N, 1, 0))])
    rho0 = H.random_rho(N)
    got = engine.propagate(sysd, grid, rho0, ops, tr)
    ref = oracle.propagate(sysd, grid, rho0, ops, tr)
    for a, b in zip(got, ref):
        assert a.shape == b.shape == (b.shape[0], 100)
        assert rel(a, b) < 1e-12
        assert np.all(np.abs(a[:, 64:]) > 0)


@pytest.mark.parametrize("fp4", ["0", "1"])
def test_free_propagator_kernel_switch_takes_effect_per_call(monkeypatch, fp4):
    """PQD_FP4 is read per plan, so both settings run their own kernel within one process (bit patterns differ in
    the last place between the packed 4x4 kernel and the general one, both match the oracle)"""
    monkeypatch.setenv("PQD_FP4", fp4)
    sysd, grid = H.random_system(2, n_steps=40, seed=12)
    got = engine.free_propagators(sysd, grid)
    assert rel(got, oracle.free_propagators(sysd, grid)) < 1e-12


def test_free_propagators_beyond_32bit_dispatch_general_kernel():
    """the general one-workgroup-per-matrix kernel at N = 3: 1700 identical systems x 2 x 5000 half steps = 17 M
    matrices x 256 threads > 2^32 work-items; the capped grid must still build every matrix"""
    N, n_sys, n_steps = 3, 1700, 5000
    sysd, grid = H.random_system(N, n_chan=1, n_lind=1, seed=6, n_steps=n_steps)
    tr = Trajectories(np.full(n_sys, n_steps - 1), np.full(n_sys, n_steps))
    tr.system = np.arange(n_sys)
    out = engine.propagate([sysd] * n_sys, grid, H.ketbra(N, 0, 0), [H.ketbra(N, 1, 1), H.ketbra(N, 0, 2)], tr)
    ref = out[0]
    assert np.all(np.isfinite(ref)) and np.abs(ref).max() > 0
    for k in (1, n_sys // 2, n_sys - 1):
        np.testing.assert_array_equal(out[k], ref)


def test_plan_timing_ring_bounded():
    """events are created once per plan and reused: many executes without a timing reset keep working"""
    sysd, grid = H.random_system(2, n_steps=5, seed=1)
    tr = Trajectories(np.array([0]), np.array([5]))
    plan = engine.Plan(sysd, grid, H.ketbra(2, 0, 0), [np.eye(2)], tr)
    for _ in range(150):
        plan.execute()
    plan.synchronize()
    f, w, n = plan.timing(reset=True)
    assert n == 64 and f >= 0 and w >= 0
    plan.execute()
    assert plan.timing(reset=False)[2] == 1


@pytest.mark.parametrize("N,n_sub", [(2, 1), (2, 2), (3, 1), (4, 1), (6, 1)])
def test_idle_half_steps_copy_the_idle_propagator(monkeypatch, N, n_sub):
    """half steps whose pulse samples are all exactly zero copy exp(L0 w)^n_sub (built once per system): same
    values as computing them (PQD_IDLE=0), and the oracle's"""
    sysd, grid = H.random_system(N, n_steps=40, n_sub=n_sub, seed=7 + N)
    chans = []
    for X, f in sysd.channels:
        f = np.array(f)
        f[: len(f) // 4] = 0.0          # drive off at the start ...
        f[len(f) // 2:] = 0.0           # ... and after the middle
        chans.append((X, f))
    sysd.channels = chans
    got = engine.free_propagators(sysd, grid)
    assert rel(got, oracle.free_propagators(sysd, grid)) < 1e-12
    monkeypatch.setenv("PQD_IDLE", "0")
    assert np.array_equal(got, engine.free_propagators(sysd, grid))
    tr = Trajectories(np.array([0, 3]), np.array([40, 38]), [MTO(1, 25, False, 1, H.ketbra(N, 1, 0))])
    ops = [H.ketbra(N, 1, 1), H.ketbra(N, 0, 1)]
    rho0 = H.random_rho(N)
    ref = oracle.propagate(sysd, grid, rho0, ops, tr)
    monkeypatch.setenv("PQD_IDLE", "1")
    for a, b in zip(engine.propagate(sysd, grid, rho0, ops, tr), ref):
        assert rel(a, b) < 1e-12
