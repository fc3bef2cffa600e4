"""Gaussian-bath PT generator (pyaceqd_amd/ptgen.py; replaces ACE's `write_PT`, general_system.py:152-211).

ACE is absent, so parity with ACE's PT files is unpinned. The generator is pinned by:
  * the closed-form independent-boson coherence (the eta_k quadrature and sign/polaron-shift conventions);
  * the exact uncompressed shift-register PT of oracle/ptgen_oracle.py with driving and Lindblad terms (the MPS
    compression, the s+/s- split step, the trace-adapted basis and the stationary repeated slice).
Propagation here runs through the C oracle (CPU); the GPU runs the same PTs in tests/test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

from oracle import oracle, ptgen_oracle
from pyaceqd_amd import ptgen
from pyaceqd_amd.constants import hbar
from pyaceqd_amd.engine import Grid, System, Trajectories
from tests import helpers as H

QDJ = lambda w: ptgen.qd_phonon_J(w, ae=3.0)  # noqa: E731


def test_qd_J_small_omega_and_units():
    """J ~ w^3 (D_e - D_h)^2 / (4 pi^2 rho hbar c^5) for w -> 0, in 1/ps"""
    w = np.array([1e-4, 2e-4])
    pref = (ptgen.QD_DE - ptgen.QD_DH) ** 2 * 1.602176634e-19 ** 2 / (
        4 * np.pi ** 2 * ptgen.QD_RHO * 1.054571817e-34 * ptgen.QD_CS ** 5) * 1e36 * 1e-12
    assert np.allclose(QDJ(w) / w ** 3, pref, rtol=1e-6)
    assert QDJ(np.array([0.0]))[0] == 0.0
    # the Gaussian form factor cuts J off above ~ 2 c_s / a
    assert QDJ(np.array([12.0]))[0] < 1e-3 * QDJ(np.array([2.0]))[0]


def test_eta_reproduces_closed_form_ibm():
    """sum of the discretised eta_k = the continuous double integral of C(t) (pure dephasing is exact at any dt)"""
    dt, K, T = 0.1, 40, 4.0
    eta, delta = ptgen.eta_coefficients(QDJ, T, dt, K)
    disc = ptgen_oracle.ibm_coherence_discrete(eta, delta, dt, K)
    exact = ptgen_oracle.ibm_coherence_exact(QDJ, T, dt * np.arange(K + 1))
    assert np.max(np.abs(disc - exact)) < 1e-9
    # the coherence drops to the Franck-Condon value |<B>|^2 and stays there; the polaron shift is removed
    assert 0.3 < abs(disc[-1]) < 0.5 and abs(np.angle(disc[-1])) < 1e-3


def test_polaron_shift_and_zero_temperature():
    eta0, d0 = ptgen.eta_coefficients(QDJ, 0.0, 0.1, 5)
    eta4, d4 = ptgen.eta_coefficients(QDJ, 4.0, 0.1, 5)
    assert d0 == d4 > 0                                   # Delta = int J/w is temperature independent
    assert np.allclose(eta0.imag, eta4.imag)              # the dissipative part does not depend on T
    assert np.all(eta4[1:].real >= eta0[1:].real - 1e-15)


@pytest.mark.parametrize("lam,K,n_init", [([0, 1], 3, 9), ([0, 1, 1], 2, 4), ([0, 1, 1, 2], 2, 7), ([0, 2], 1, 2)])
def test_generator_matches_exact_shift_register(lam, K, n_init):
    """driven, damped N-level system with a 30x enhanced bath: compressed generator (threshold 1e-14, explicit
    slices then the repeated stationary slice) vs the exact shift-register PT over 40 steps"""
    N = len(lam)
    A = np.diag(np.array(lam, dtype=float))
    J = lambda w: 30 * QDJ(w)  # noqa: E731
    eta, delta = ptgen.eta_coefficients(J, 4.0, 0.1, K)
    sysd, grid = H.random_system(N, n_steps=40, seed=3 + N)
    rho0 = H.random_rho(N)
    ops = [H.ketbra(N, i, j) for i in range(N) for j in range(N)]
    tr = Trajectories(np.array([0, 5]), np.array([40, 33]))
    pg = ptgen.build_gaussian_pt(A, 0.1, eta, delta, threshold=1e-14, max_bond=0, n_init=n_init)
    pe = ptgen_oracle.exact_if_pt(A, eta, delta, 0.1)
    assert pg.chi <= pe.chi
    got = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pg)
    ref = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pe)
    bare = oracle.propagate(sysd, grid, rho0, ops, tr)
    for a, b, c in zip(got, ref, bare):
        assert np.max(np.abs(a - b)) < 1e-11
        assert np.max(np.abs(b - c)) > 1e-2        # the bath matters at this coupling


def test_generated_pt_ibm_long_run():
    """QD phonons, K = 8, threshold 1e-8: coherence vs the discretised IBM solution for 8K steps (2K explicit
    slices, then the repeated slice), trace preserved. The truncation error grows ~ threshold per step."""
    dt, K = 0.1, 8
    eta, delta = ptgen.eta_coefficients(QDJ, 4.0, dt, K)
    pt = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), dt, eta, delta, threshold=1e-8, max_bond=0)
    n = 8 * K
    out = oracle.propagate(System(dim=2, H0=np.zeros((2, 2))), Grid(0.0, dt, n), 0.5 * np.ones((2, 2), complex),
                           [H.ketbra(2, 0, 1), np.eye(2)], Trajectories(np.array([0]), np.array([n])), pt=pt)[0]
    ex = ptgen_oracle.ibm_coherence_discrete(eta, delta, dt, n)
    assert np.max(np.abs(out[:, 0] - ex)) < 1e-5
    assert np.max(np.abs(out[:, 1] - 1)) < 1e-9


def test_bond_cap_and_padding():
    eta, delta = ptgen.eta_coefficients(QDJ, 4.0, 0.1, 8)
    pt = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), 0.1, eta, delta, threshold=1e-12, max_bond=16)
    assert pt.chi == 16 and pt.n_init == 16 and pt.n_slices == 17
    assert pt.D == 4 and list(pt.gmap) == [0, 1, 2, 3]


def test_truncation_record_says_when_the_cap_decided():
    """every generated PT records what set its boundary cuts (pt.meta['truncation']): with a
    cap below the threshold's rank the cap decided (warning raised, the largest discarded singular value far above
    the threshold); without a cap the threshold decided every cut (largest discarded value <= threshold)"""
    import warnings
    eta, delta = ptgen.eta_coefficients(QDJ, 4.0, 0.1, 8)
    with pytest.warns(RuntimeWarning, match="bond cap 16"):
        capped = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), 0.1, eta, delta, threshold=1e-12, max_bond=16)
    tc = capped.meta["truncation"]
    assert tc["cap_decided"] and tc["cap_bound"] > 0 and tc["max_rank_wanted"] > 16
    assert tc["max_discarded_rel"] > 1e-12
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        free = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), 0.1, eta, delta, threshold=1e-8, max_bond=0)
    tf = free.meta["truncation"]
    assert not tf["cap_decided"] and tf["cap_bound"] == 0 and tf["compressions"] == 2 * (2 * 8 + 1)
    assert 0 < tf["max_discarded_rel"] <= 1e-8


def test_driver_generates_and_caches_pt(tmp_path, monkeypatch):
    """system_ace_stream(phonons=True) without a PT file: generate from the ACE generate-file parameters, cache
    under the reference's name (+ .npz), reuse on the next call; J_to_file writes J(omega). (The driver generates on
    the GPU by default; this CPU test takes the host restatement, PQD_PTGEN=host: tests/test_gpu_ptgen.py runs the
    default.)"""
    monkeypatch.setenv("PQD_PTGEN", "host")
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd import opgrammar
    B = opgrammar.to_matrix("1.000*|1><1|_2", 2)
    kw = dict(dt=0.1, t_mem=0.5, ae=3.0, temperature=4, threshold="9", factor_ah=None, boson_e_max=7, J_file=None,
              J_to_file=None, use_infinite=True, system_prefix="tls", temp_dir=str(tmp_path) + os.sep, verbose=False)
    pt = gs._resolve_pt(None, B, **kw)
    name = str(tmp_path / ptgen.pt_cache_name("tls", 3.0, 4, "9", 0.5, 0.1, use_infinite=True)) + ".npz"
    assert os.path.isfile(name)
    pt2 = gs._resolve_pt(None, B, **kw)
    # use_infinite: the memory is the bath's own, bounded by the te = 2 t_mem horizon (20 steps here, not converged at
    # a_e = 3 nm), not round(t_mem / dt) = 5
    assert np.array_equal(pt.Q, pt2.Q) and pt.meta["K"] == 10 and pt.n_init == 20
    jf = str(tmp_path / "J.dat")
    gs._write_J(jf, 3.0, None, None)
    d = np.loadtxt(jf)
    assert d.shape == (2000, 2) and abs(d[-1, 0] - 15 / hbar) < 1e-9
    assert np.allclose(d[:, 1], QDJ(d[:, 0]))
    # J_file round trip
    J2 = ptgen.J_from_file(jf)
    w = np.linspace(0.5, 5, 7)
    assert np.allclose(J2(w), QDJ(w), rtol=2e-3)


def test_driver_falls_back_when_ace_file_layout_unknown(tmp_path, monkeypatch):
    """An existing `<pt_file>_initial` in a layout the ACE reader does not know (e.g. one ACE itself wrote) is not
    an error of the call: the driver warns and takes the pqd PT (generated and cached here), as it would with no ACE
    file present (general_system.py _resolve_pt)"""
    import warnings
    monkeypatch.setenv("PQD_PTGEN", "host")
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd import opgrammar
    B = opgrammar.to_matrix("1.000*|1><1|_2", 2)
    kw = dict(dt=0.1, t_mem=0.3, ae=3.0, temperature=4, threshold="9", factor_ah=None, boson_e_max=7, J_file=None,
              J_to_file=None, use_infinite=True, system_prefix="tls", temp_dir=str(tmp_path) + os.sep, verbose=False)
    name = str(tmp_path / ptgen.pt_cache_name("tls", 3.0, 4, "9", 0.3, 0.1, use_infinite=True))
    for suf in ("_initial", "_initial_0", "_repeated", "_repeated_0"):
        with open(name + suf, "wb") as f:
            f.write(b"\x00\x01not a layout this reader knows\n")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        pt = gs._resolve_pt(None, B, **kw)
    assert any("not in a layout" in str(x.message) for x in w)
    assert pt.n_init == 12 and os.path.isfile(name + ".npz")   # use_infinite: K = 2 t_mem / dt = 6 (horizon)


# ------------------------------------------------------------------ use_infinite and PT provenance
def _influence(pt, paths):
    out = []
    for path in paths:
        v = pt.bond0.copy()
        s = 0
        for n, a in enumerate(path):
            s = n if n < pt.n_init else pt.n_init + (n - pt.n_init) % (pt.n_slices - pt.n_init)
            v = v @ pt.Q[s, pt.gmap[a]]
        out.append(v @ pt.closure[s])
    return np.array(out)


def test_infinite_memory_steps_rule():
    """use_Gaussian_infinite (general_system.py:150-151, 165-167) takes the bath's own memory: the shortest K whose
    neglected eta_k tail is below the threshold, bounded by the generate file's te = 2 t_mem horizon. The tls default
    (tls.py:18: dt 0.1, a_e 5 nm, 4 K, threshold 1e-8) converges at K = 65 whatever t_mem; a_e = 3 nm keeps a ~1e-9
    eta floor (the hard Boson_E_max cut of J) and takes the whole horizon."""
    tls_B = np.diag([0.0, 1.0])
    for tm in (6.4, 20.48):
        _, _, info = ptgen.qd_phonon_eta(tls_B, 0.1, tm, 5.0, 4, 1e-8, use_infinite=True)
        assert info["K"] == 65 and info["converged"]
    _, _, info = ptgen.qd_phonon_eta(np.diag([0.0, 1, 1, 2]), 0.5, 20.48, 3.0, 4, 1e-10, use_infinite=True)
    assert info["K"] == 82 and not info["converged"]
    _, _, info = ptgen.qd_phonon_eta(tls_B, 0.1, 6.4, 5.0, 4, 1e-8, use_infinite=False)
    assert info["K"] == 64
    # the rule itself: the tail beyond K is below the threshold, the tail beyond K - 1 is not
    eta, _, _ = ptgen.qd_phonon_eta(tls_B, 0.1, 6.4, 5.0, 4, 1e-8, K=128)
    a = np.abs(eta)
    assert a[66:].sum() <= 1e-8 < a[65:].sum()


def test_infinite_memory_pt_converged_in_memory():
    """the use_infinite PT does not change when its memory is doubled: influence values of 300 random paths (up to
    6 K steps, explicit and repeated slices) agree to <= 10 x threshold (measured 3e-3 x threshold), while a
    memory cut at K / 3 (what a short t_mem gives) moves them by > 100 x threshold"""
    B, dt, thr = np.diag([0.0, 1.0]), 0.5, 1e-8
    kw = dict(t_mem=20.48, ae=5.0, temperature=4, threshold=thr, use_infinite=True)
    p1 = ptgen.qd_phonon_pt(B, dt, **kw)
    K = p1.meta["K"]
    assert p1.meta["converged"] and 10 <= K <= 20
    p2 = ptgen.qd_phonon_pt(B, dt, K=2 * K, **kw)
    p3 = ptgen.qd_phonon_pt(B, dt, K=K // 3, **kw)
    rng = np.random.default_rng(0)
    paths = [rng.integers(0, 4, size=rng.integers(1, 6 * K)) for _ in range(300)]
    a, b, c = _influence(p1, paths), _influence(p2, paths), _influence(p3, paths)
    assert np.max(np.abs(a - b)) <= 10 * thr * np.max(np.abs(b))
    assert np.max(np.abs(c - b)) > 100 * thr * np.max(np.abs(b))


def _kw(tmp_path, **over):
    kw = dict(dt=0.5, t_mem=2.0, ae=5.0, temperature=4, threshold="7", factor_ah=None, boson_e_max=7, J_file=None,
              J_to_file=None, use_infinite=True, system_prefix="tls", temp_dir=str(tmp_path) + os.sep, verbose=False)
    kw.update(over)
    return kw


def test_cached_pt_regenerated_when_parameters_differ(tmp_path, monkeypatch):
    """the reference's use_infinite cache name leaves out a_e (general_system.py:150-151): a second call at another
    a_e finds the first call's file. Its stored generation parameters differ, so it is regenerated (with a warning)
    and replaced; a third call at the same parameters reuses it silently"""
    import warnings
    monkeypatch.setenv("PQD_PTGEN", "host")
    from pyaceqd_amd.general_system import general_system as gs
    B = np.diag([0.0, 1.0]).astype(complex)
    p5 = gs._resolve_pt(None, B, **_kw(tmp_path, ae=5.0))
    assert p5.meta["ae"] == 5.0 and p5.meta["generator"] == "host" and p5.meta["dt"] == 0.5
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        p4 = gs._resolve_pt(None, B, **_kw(tmp_path, ae=4.0))
    assert any("regenerating" in str(x.message) and "'ae'" in str(x.message) for x in w)
    path = [np.full(12, 2)]
    assert p4.meta["ae"] == 4.0 and abs(_influence(p4, path)[0] - _influence(p5, path)[0]) > 1e-3
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        p4b = gs._resolve_pt(None, B, **_kw(tmp_path, ae=4.0))
    assert not w and np.array_equal(p4b.Q, p4.Q)
    # the bond cap and the threshold are part of the key as well
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        gs._resolve_pt(None, B, **_kw(tmp_path, ae=4.0, threshold="8"))
    assert not any("regenerating" in str(x.message) for x in w)     # another threshold has another file name
    from pyaceqd_amd.pt import load_pt, save_pt
    name = [f for f in os.listdir(tmp_path) if f.endswith("th7_dt0.5.pt.npz")][0]
    p = load_pt(str(tmp_path / name))
    p.meta["max_bond"] = 64
    save_pt(str(tmp_path / name), p, dim=2)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        gs._resolve_pt(None, B, **_kw(tmp_path, ae=4.0))
    assert any("regenerating" in str(x.message) and "max_bond" in str(x.message) for x in w)


def test_pt_dt_and_dimension_mismatch_raise(tmp_path, monkeypatch):
    """a PT generated at dt = 0.5 handed to a dt = 0.1 run, or a two-level PT to a four-level run, is an error
    (ValueError), whether named explicitly, found in the cache or passed as an object"""
    monkeypatch.setenv("PQD_PTGEN", "host")
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd.pt import save_pt
    B = np.diag([0.0, 1.0]).astype(complex)
    p = gs._resolve_pt(None, B, **_kw(tmp_path))
    f = str(tmp_path / "mine.npz")
    save_pt(f, p, dim=2)
    with pytest.raises(ValueError, match="dt = 0.5"):
        gs._resolve_pt(f, B, **_kw(tmp_path, dt=0.1))
    with pytest.raises(ValueError, match="dt = 0.5"):
        gs._resolve_pt(p, B, **_kw(tmp_path, dt=0.1))
    with pytest.raises(ValueError, match="Liouville rows"):
        gs._resolve_pt(f, np.diag([0.0, 1, 1, 2]).astype(complex), **_kw(tmp_path))
    # explicitly named: used as given even when the stored parameters differ (the reference uses a given pt_file)
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        q = gs._resolve_pt(f, B, **_kw(tmp_path, ae=3.0))
    assert np.array_equal(q.Q, p.Q) and any("used as given" in str(x.message) for x in w)


def test_explicit_unreadable_ace_file_raises(tmp_path, monkeypatch):
    """an explicitly named ACE PT (`<pt_file>_initial`) in a layout this reader does not know is an error: it may
    hold another bath, so no PT is generated in its place; under the automatic name the driver warns and
    generates (test_driver_falls_back_when_ace_file_layout_unknown)"""
    monkeypatch.setenv("PQD_PTGEN", "host")
    from pyaceqd_amd.general_system import general_system as gs
    name = str(tmp_path / "user_pt")
    for suf in ("_initial", "_initial_0", "_repeated", "_repeated_0"):
        with open(name + suf, "wb") as f:
            f.write(b"\x00\x01not a layout this reader knows\n")
    with pytest.raises(ValueError, match="named explicitly"):
        gs._resolve_pt(name, np.diag([0.0, 1.0]).astype(complex), **_kw(tmp_path))
