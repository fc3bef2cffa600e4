"""two_time/correlations.py against the reference's OWN functions.

tests/golden/pyref_correlations.npz: the reference `two_op_one_time`, `three_op_one_time`, `two_op_two_time`,
`three_op_two_time` (t_start 0 and < 0), `five_op_two_time`, and `tl_two_op_two_time` / `tl_three_op_two_time` in
all three branches (use_dm x fortran_only), run on tests/fake_system.py with the reference Fortran behind
propagate_tau_module (tests/golden/make_golden.py gen_correlations).

tests/golden/pyref_twotime_anchor.npz: the reference tl_three_op_two_time / tl_two_op_two_time (use_dm=True) fed with
exact no-phonon dynamical maps of a driven biexciton (make_golden.py gen_twotime_anchor). Our TRAJECTORY sweep
(three_op_two_time / two_op_two_time: MTOs applied at t1 inside the propagation) must reproduce them: this pins the
two-time semantics of the PT path (MTO timing and sides, output slicing) to the reference's map formula.

CPU tests route the two GPU kernels these paths use (calc_tl_dynmap_pseudo's batched pinv, the map-chain sweep) and
the propagation through the CPU oracle; the `gpu` tests run the same calls on libpqd.
"""
import os

import numpy as np
import pytest

from pyaceqd_amd.pulses import ChirpedPulse
from pyaceqd_amd.two_time import correlations as corr
from tests.fake_system import fake_system, fake_system_dm

TOL = 1e-12


def close(a, b, tol=TOL):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))
    assert err < tol, err


@pytest.fixture(scope="module")
def z(golden_dir):
    return np.load(os.path.join(golden_dir, "pyref_correlations.npz"))


@pytest.fixture(scope="module")
def anchor(golden_dir):
    return np.load(os.path.join(golden_dir, "pyref_twotime_anchor.npz"))


def _p():
    return ChirpedPulse(tau_0=1.0, e_start=0, e0=1.5, t0=2)


def _opts(**k):
    return dict({"lindblad": True, "phonons": False}, **k)


def _oracle_kernels(monkeypatch):
    """CPU stand-ins for the GPU kernels of the map paths (test infrastructure only)"""
    from oracle import oracle
    from pyaceqd_amd.two_time import propagate_tau_module as ptm
    monkeypatch.setattr(corr, "calc_tl_dynmap_pseudo", lambda dm, t, debug=False: oracle.tl_dynmap_pseudo(
        np.asarray(dm)[: len(t) - 1]))
    monkeypatch.setattr(ptm, "calc_onetime_parallel", lambda dm, r, n_tau, dim, a, b, c, t, ts: oracle.
                        calc_onetime_parallel(dm, r, n_tau, dim, a, b, c, np.real(t), ts))
    monkeypatch.setattr(ptm, "map_tail", oracle.map_tail)


def _oracle_propagation(monkeypatch):
    from oracle import oracle
    import pyaceqd_amd._lib as L
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd.engine import tables_from_outputs
    monkeypatch.setattr(L, "context", lambda device=None: None)
    monkeypatch.setattr(gs, "propagate", lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None: oracle.propagate(
        system, grid, rho0, out_ops, traj, pt=pt, nthreads=4))
    monkeypatch.setattr(gs, "propagate_table", lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None:
                        tables_from_outputs(oracle.propagate(system, grid, rho0, out_ops, traj, pt=pt, nthreads=4),
                                            traj, grid))


# ------------------------------------------------------------------------------------------- trajectory drivers
def test_one_time_drivers_match_reference(z):
    tau, G = corr.two_op_one_time(fake_system, _p(), opA="|1><0|_2", opB="|0><1|_2", t0=-2, t_MTO=1.0, tend=4, dt=0.1,
                                  options=_opts())
    close(tau, z["ot2_tau"]); close(G, z["ot2_G"])
    tau, G = corr.three_op_one_time(fake_system, _p(), t0=-2, t_MTO=1.0, tend=4, dt=0.1, options=_opts())
    close(tau, z["ot3_tau"]); close(G, z["ot3_G"])


@pytest.mark.parametrize("tag,name,kw", [("tt2", "two_op_two_time", {}), ("tt3", "three_op_two_time", {}),
                                         ("tt3s", "three_op_two_time", {"t_start": -1.0}),
                                         ("tt5", "five_op_two_time", {"t_start": -1.0})])
def test_two_time_drivers_match_reference(z, tag, name, kw):
    """_ops_two_time (correlations.py:135-184): one batched launch for all t1 vs one system call per t1"""
    t1, t2, G = getattr(corr, name)(fake_system, z["t_axis"], _p(), tau_max=2.0, dt=0.1, options=_opts(), workers=2,
                                    **kw)
    close(t1, z[f"{tag}_t1"]); close(t2, z[f"{tag}_t2"]); close(G, z[f"{tag}_G"])


# ------------------------------------------------------------------------------------------- time-local-map paths
BRANCHES = [(False, False), (True, False), (True, True)]
RHO2 = np.array([[0.8, 0.1 - 0.05j], [0.1 + 0.05j, 0.2]], dtype=complex)


def _rho4():
    r = np.diag([0.5, 0.2, 0.2, 0.1]).astype(complex)
    r[0, 3] = r[3, 0] = 0.05
    return r


def _tl_cases(z):
    for use_dm, fo in BRANCHES:
        key = f"dm{int(use_dm)}_f{int(fo)}"
        yield (f"tl2_{key}", lambda u=use_dm, f=fo: corr.tl_two_op_two_time(
            fake_system_dm, z["t_axis"], _p(), t_mem=1.0, tau_max=2.0, dt=0.1, rho0=RHO2, options=_opts(), use_dm=u,
            fortran_only=f))
        yield (f"tl3_{key}", lambda u=use_dm, f=fo: corr.tl_three_op_two_time(
            fake_system_dm, z["t_axis"], _p(), t_mem=1.0, opC="|0><1|_2", tau_max=2.0, dt=0.1, rho0=RHO2,
            options=_opts(), use_dm=u, fortran_only=f))
        yield (f"tl3d4_{key}", lambda u=use_dm, f=fo: corr.tl_three_op_two_time(
            fake_system_dm, z["t_axis"], _p(), t_mem=1.0, opA="|1><0|_4", opB="|2><1|_4", opC="|3><1|_4",
            tau_max=1.5, dt=0.1, rho0=_rho4(), options=_opts(fake_dim=4), use_dm=u, fortran_only=f))


def test_tl_paths_match_reference_cpu(z, monkeypatch):
    """all branches of tl_two_op_two_time / tl_three_op_two_time, kernels on the CPU oracle"""
    _oracle_kernels(monkeypatch)
    for key, run in _tl_cases(z):
        _, t2, G = run()
        close(G, z[key + "_G"], 1e-10)


def test_tl_three_op_stationary_opt_in_differs(z, monkeypatch):
    """the reference's non-dm tl_three_op_two_time ignores opC (its two-op formula); the opt-in three-op form does not"""
    _oracle_kernels(monkeypatch)
    _, _, G = corr.tl_three_op_two_time(fake_system_dm, z["t_axis"], _p(), t_mem=1.0, opC="|0><1|_2", tau_max=2.0,
                                        dt=0.1, rho0=RHO2, options=_opts(), three_op_stationary=True)
    assert np.max(np.abs(G - z["tl3_dm0_f0_G"])) > 1e-3
    with pytest.raises(ValueError):
        corr.tl_three_op_two_time(fake_system_dm, z["t_axis"], _p(), t_mem=1.0, rho0=RHO2, options=_opts(),
                                  use_dm=True, three_op_stationary=True)


@pytest.mark.gpu
def test_tl_paths_match_reference_gpu(z):
    """the same calls with the GPU pinv and the GPU map-chain sweep"""
    for key, run in _tl_cases(z):
        _, t2, G = run()
        close(G, z[key + "_G"], 1e-10)


# ------------------------------------------------------------------------------------------- PT-path anchor
def _anchor_runs(anchor):
    from pyaceqd_amd.four_level_system.linear import biexciton
    p = ChirpedPulse(tau_0=1.0, e_start=-2.0, e0=1.3, t0=1.5, polar_x=0.8)
    opts = lambda: {"lindblad": True, "phonons": False, "delta_b": 4.0, "delta_xy": 0.03}  # noqa: E731
    t_axis = anchor["t_axis"]
    _, tau, G2 = corr.three_op_two_time(biexciton, t_axis, p, opA="|3><1|_4", opB="|1><1|_4", opC="|1><3|_4",
                                        tau_max=4.0, dt=0.1, options=opts())
    _, _, G1 = corr.two_op_two_time(biexciton, t_axis, p, opA="|1><0|_4", opB="|0><1|_4", tau_max=4.0, dt=0.1,
                                    options=opts())
    return tau, G2, G1


def _check_anchor(anchor, tau, G2, G1):
    close(tau, anchor["tau"])
    close(G2, anchor["g2_f1"], 1e-10)   # the reference's Fortran sweep (column-major view; A = C^T, B = B^T here)
    close(G2, anchor["g2_f0"], 1e-10)   # the reference's row-major Python sweep
    close(G1, anchor["g1_f0"], 1e-10)


def test_trajectory_sweep_matches_reference_map_formula_cpu(anchor, monkeypatch):
    """our batched trajectory sweep's host bookkeeping on the CPU oracle vs the reference's map-based G2 / G1"""
    _oracle_propagation(monkeypatch)
    _check_anchor(anchor, *_anchor_runs(anchor))


@pytest.mark.gpu
def test_trajectory_sweep_matches_reference_map_formula_gpu(anchor):
    """the HIP sweep (MTOs at t1 in the kernel) vs the reference's map-based G2 / G1 on the same biexciton"""
    _check_anchor(anchor, *_anchor_runs(anchor))


# ------------------------------------------------------------------------------------------- spectrum, phonon maps
@pytest.fixture(scope="module")
def zph(golden_dir):
    return np.load(os.path.join(golden_dir, "pyref_correlations_phonons.npz"))


def test_get_spectrum_matches_reference(zph):
    """reference get_spectrum (correlations.py:322-380) on an analytic two-line G1 with an offset"""
    s, om = corr.get_spectrum(zph["sp_g1"], zph["sp_tau"])
    close(om, zph["sp_omega"])
    close(s, zph["sp_s"])


def _phonon_map_call(fn, zph):
    return fn(fake_system_dm, zph["ph_t_axis"], _p(), t_mem=1.0, tau_max=50.0, dt=0.1,
              rho0=np.array([[0.8, 0.1 - 0.05j], [0.1 + 0.05j, 0.2]], dtype=complex), opB="|0><0|_2",
              options={"lindblad": True, "phonons": True, "output_ops": ["|0><0|_2", "|1><1|_2"]})


@pytest.mark.parametrize("name,tag", [("tl_three_op_two_time_phonons", "ph"),
                                      ("tl_threeoptwotime_phonons_dm", "phdm")])
def test_phonon_map_correlations_match_reference(monkeypatch, zph, name, tag):
    """reference tl_three_op_two_time_phonons (:866-1011) / tl_threeoptwotime_phonons_dm (:1013-1186) on the
    calc_dynmap fake model: t < t_mem rows from per-t dynamical-map runs, later rows from the 1.2 t_mem run, tails
    on the last time-local map (the GPU batched pinv replaced by the oracle here; tests/test_gpu_parity.py runs it)"""
    _oracle_kernels(monkeypatch)
    t, tau, G = _phonon_map_call(getattr(corr, name), zph)
    close(tau, zph[f"{tag}_tau"])
    close(G, zph[f"{tag}_G"], 1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("name,tag", [("tl_three_op_two_time_phonons", "ph"),
                                      ("tl_threeoptwotime_phonons_dm", "phdm")])
def test_phonon_map_correlations_match_reference_gpu(zph, name, tag):
    """the same with the time-local maps from the GPU batched pinv (tlmap.hip)"""
    t, tau, G = _phonon_map_call(getattr(corr, name), zph)
    close(G, zph[f"{tag}_G"], 1e-10)
