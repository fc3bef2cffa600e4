"""The C restatement of the reference's Fortran sweeps (oracle/mapchain_oracle.c) against golden vectors
produced by the reference Fortran itself (tests/golden/fortran_*.npz, made by tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from oracle import oracle

F = lambda maps: np.asfortranarray(np.asarray(maps).transpose(1, 2, 0))  # noqa: E731
TOL = 1e-12


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def rel(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b)))


@pytest.mark.parametrize("dim", [2, 4, 6])
def test_propagate_tau(golden_dir, dim):
    z = load(golden_dir, f"fortran_propagate_tau_d{dim}.npz")
    r = oracle.propagate_tau(F(z["dm_tl"]), z["rho_init"], int(z["n_tau"]), dim, int(z["j_start"]))
    assert rel(r, z["rho_out"]) < TOL


@pytest.mark.parametrize("dim", [2, 4, 6])
def test_calc_onetime_parallel(golden_dir, dim):
    z = load(golden_dir, f"fortran_onetime_d{dim}.npz")
    r = oracle.calc_onetime_parallel(F(z["dm_tl"]), z["rho_init"], int(z["n_tau"]), dim, z["opa"], z["opb"], z["opc"],
                                     z["time"], z["time_sparse"], nthreads=2)
    assert rel(r, z["result"]) < TOL


@pytest.mark.parametrize("dim", [2, 4, 6])
def test_calc_onetime_parallel_block(golden_dir, dim):
    z = load(golden_dir, f"fortran_onetime_block_d{dim}.npz")
    r = oracle.calc_onetime_parallel_block(F(z["dm_block"]), z["dm_s"], z["rho_init"], int(z["n_tb"]),
                                           int(z["nx_tau"]), dim, z["opa"], z["opb"], z["opc"], z["time"],
                                           z["time_sparse"])
    assert rel(r, z["result"]) < TOL


@pytest.mark.parametrize("dim", [2, 4, 6])
def test_calc_twotime_phonon_block(golden_dir, dim):
    z = load(golden_dir, f"fortran_twotime_phonon_block_d{dim}.npz")
    dtc = np.asfortranarray(z["dm_taucs2"].transpose(2, 3, 0, 1))
    r = oracle.calc_twotime_phonon_block(dtc, F(z["dm_sep1"]), F(z["dm_sep2"]), z["dm_s"], z["rho_init"],
                                         int(z["n_tb"]), int(z["nx_tau"]), dim, z["opa"], z["opb"], z["opc"],
                                         z["time"], z["time_sparse"])
    assert rel(r, z["result"]) < TOL


@pytest.mark.parametrize("dim", [2, 4, 5])
def test_timebin(golden_dir, dim):
    z = load(golden_dir, f"fortran_timebin_d{dim}.npz")
    args = (F(z["dm_1"]), F(z["dm_2"]), z["rho_init"], z["t1"], F(z["precalc"]), float(z["dt"]), dim)
    ops8 = list(z["ops8"])
    assert rel(oracle.four_time_8op(*args, ops8, False, False, float(z["tb"])), z["result8"]) < TOL
    assert rel(oracle.four_time_8op(*args, ops8, True, False, float(z["tb"])), z["result8_early"]) < TOL
    assert rel(oracle.four_time_8op(*args, ops8, False, True, float(z["tb"])), z["result8_late"]) < TOL
    assert rel(oracle.four_time(*args, ops8[:4], float(z["tb"])), z["result4"]) < TOL
    assert rel(oracle.dynamics_t1(*args, float(z["tb"])), z["dyn_t1"]) < TOL


def test_fortran_ref_live_if_built():
    """Where oracle/_ref was built from the reference sources, re-check on fresh random inputs."""
    from oracle import fref
    if not fref.available():
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(5)
    dim, n_tfull, n_tau = 3, 40, 15
    N2 = dim * dim
    maps = (np.eye(N2) + 0.1 * (rng.normal(size=(n_tfull - 1, N2, N2)) + 1j * rng.normal(size=(n_tfull - 1, N2, N2))))
    rho = rng.normal(size=N2) + 1j * rng.normal(size=N2)
    ops = [rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)) for _ in range(3)]
    time = np.round(np.arange(n_tfull) * 0.2, 6)
    ts = np.array([0.0, 0.2, 0.5, 1.3, 2.2])
    a = fref.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts)
    b = oracle.calc_onetime_parallel(F(maps), rho, n_tau, dim, *ops, time, ts)
    assert rel(b, a) < TOL
