"""Generate the committed golden fixtures under tests/golden/.

Run in the build container only (needs /root/reference and oracle/_ref built by `make -C oracle ref`):
    python tests/golden/make_golden.py

Two kinds of vectors, both produced by running the REFERENCE ITSELF on seeded inputs:
  * fortran_*.npz : outputs of the reference Fortran sweep kernels
                    (pyaceqd/two_time/propagate_tau.f90, pyaceqd/timebin/timebin_tl.f90), compiled from
                    their own sources by oracle/Makefile and called through oracle/fref.py.
  * pyref_*.npz   : outputs of the reference's pure-Python modules that import without ACE
                    (pyaceqd/pulses.py, pyaceqd/tools.py), imported from /root/reference.
Inputs are synthetic (numpy default_rng seeds below), stored next to the outputs.
"""
import os
import sys

import numpy as np
import scipy.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import fref  # noqa: E402

REF_ROOT = "/root/reference"


def rand_lindblad_maps(n, dim, h, rng, drift=0.05):
    """n CPTP maps exp(L_i h) (row-major vec convention) of random Lindbladians that drift with i."""
    N2 = dim * dim
    I = np.eye(dim)
    H = rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)); H = 0.5 * (H + H.conj().T)
    dH = rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim)); dH = 0.5 * (dH + dH.conj().T)
    Ls = [(rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) * 0.3 for _ in range(2)]
    maps = np.empty((n, N2, N2), dtype=np.complex128)
    for i in range(n):
        Hi = H + drift * np.sin(0.1 * i) * dH
        L = -1j * (np.kron(Hi, I) - np.kron(I, Hi.T))
        for Lk in Ls:
            LdL = Lk.conj().T @ Lk
            L = L + np.kron(Lk, Lk.conj()) - 0.5 * np.kron(LdL, I) - 0.5 * np.kron(I, LdL.T)
        maps[i] = sla.expm(L * h)
    return maps


def rand_op(dim, rng):
    return rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))


def rand_rho(dim, rng):
    A = rand_op(dim, rng)
    r = A @ A.conj().T
    return r / np.trace(r)


def F(maps):
    """(n, N2, N2) row-major stack -> Fortran (N2, N2, n) layout as the reference callers build it
    (correlations.py:781 `np.asfortranarray(dm_tl.transpose(1, 2, 0))`)."""
    return np.asfortranarray(maps.transpose(1, 2, 0))


def gen_fortran():
    out = {}
    for dim in (2, 4, 6):
        rng = np.random.default_rng(1000 + dim)
        N2 = dim * dim
        # --- propagate_tau (propagate_tau.f90:3)
        maps = rand_lindblad_maps(60, dim, 0.1, rng)
        rho0 = rand_rho(dim, rng).reshape(N2)
        n_tau, j_start = 25, 7
        r = fref.propagate_tau(F(maps), rho0, n_tau, dim, j_start)
        np.savez_compressed(os.path.join(HERE, f"fortran_propagate_tau_d{dim}.npz"),
                            dm_tl=maps, rho_init=rho0, n_tau=n_tau, j_start=j_start, rho_out=np.asarray(r))
        # --- calc_onetime_parallel (propagate_tau.f90:110): time grid + sparse grid incl. off-grid values
        n_tfull = 90
        dt = 0.1
        time = np.round(np.arange(n_tfull) * dt, 6)
        time_sparse = np.array([0.0, 0.1, 0.25, 0.5, 1.0, 1.05, 2.3, 3.0, 4.4])
        n_tau = 40
        opa, opb, opc = rand_op(dim, rng), rand_op(dim, rng), rand_op(dim, rng)
        maps = rand_lindblad_maps(n_tfull - 1, dim, dt, rng)
        res = fref.calc_onetime_parallel(F(maps), rho0, n_tau, dim, opa, opb, opc, time, time_sparse)
        np.savez_compressed(os.path.join(HERE, f"fortran_onetime_d{dim}.npz"),
                            dm_tl=maps, rho_init=rho0, n_tau=n_tau, opa=opa, opb=opb, opc=opc,
                            time=time, time_sparse=time_sparse, result=np.asarray(res))
        # --- calc_onetime_parallel_block (propagate_tau.f90:189)
        n_map, n_tb, nx_tau = 6, 10, 3
        dm_block = rand_lindblad_maps(n_map, dim, dt, rng)
        dm_s = rand_lindblad_maps(1, dim, dt, rng)[0]
        time_sparse_b = np.array([0.0, 0.2, 0.35, 0.9, 1.5])
        res = fref.calc_onetime_parallel_block(F(dm_block), dm_s, rho0, n_tb, nx_tau, dim, opa, opb, opc,
                                               time, time_sparse_b)
        np.savez_compressed(os.path.join(HERE, f"fortran_onetime_block_d{dim}.npz"),
                            dm_block=dm_block, dm_s=dm_s, rho_init=rho0, n_tb=n_tb, nx_tau=nx_tau,
                            opa=opa, opb=opb, opc=opc, time=time, time_sparse=time_sparse_b, result=np.asarray(res))
        # --- calc_twotime_phonon_block (propagate_tau.f90:374)
        n_tauc = 3
        dm_sep1 = rand_lindblad_maps(n_map, dim, dt, rng)
        dm_sep2 = rand_lindblad_maps(n_map, dim, dt, rng)
        dm_tc = np.stack([rand_lindblad_maps(n_map, dim, dt, rng) for _ in range(n_tauc)])  # (n_tauc, n_map, N2, N2)
        dm_taucs2_f = np.asfortranarray(dm_tc.transpose(2, 3, 0, 1))  # purity.py:581
        time_sparse_p = np.array([0.0, 0.1, 0.2, 0.45, 0.7, 1.2])
        res = fref.calc_twotime_phonon_block(dm_taucs2_f, F(dm_sep1), F(dm_sep2), dm_s, rho0, n_tb, nx_tau, dim,
                                             opa, opb, opc, time, time_sparse_p)
        np.savez_compressed(os.path.join(HERE, f"fortran_twotime_phonon_block_d{dim}.npz"),
                            dm_taucs2=dm_tc, dm_sep1=dm_sep1, dm_sep2=dm_sep2, dm_s=dm_s, rho_init=rho0,
                            n_tb=n_tb, nx_tau=nx_tau, opa=opa, opb=opb, opc=opc, time=time,
                            time_sparse=time_sparse_p, result=np.asarray(res))
    # --- timebin_tl (timebin_tl.f90): dim 2 and 4 (dim 5 is the reference default, twophoton_new.py:19)
    for dim in (2, 4, 5):
        rng = np.random.default_rng(2000 + dim)
        N2 = dim * dim
        dt, tb = 0.1, 3.0
        n_map = 12
        dm_1 = rand_lindblad_maps(n_map, dim, dt, rng)
        dm_2 = rand_lindblad_maps(n_map, dim, dt, rng)
        tl = rand_lindblad_maps(1, dim, dt, rng)[0]
        n_precalc = int(np.log2(tb / dt)) + 1  # twophoton_new.py:606
        precalc = np.stack([np.linalg.matrix_power(tl, 2 ** k) for k in range(n_precalc)])
        # conj-transposed feed as the caller does (twophoton_new.py:114-116)
        dm_1c = np.conj(dm_1); dm_2c = np.conj(dm_2); prec_c = np.conj(precalc)
        rho0 = rand_rho(dim, rng).reshape(N2)
        # non-uniform t1 grid with a value that exercises int(round_to_6(t)/dt) truncation (0.3/0.1 -> 2)
        t1 = np.array([0.0, 0.1, 0.3, 0.6, 0.7, 1.0, 1.4, 2.0, 2.5])
        ops8 = [rand_op(dim, rng) for _ in range(8)]
        res8 = fref.four_time_8op(F(dm_1c), F(dm_2c), rho0, t1, F(prec_c), dt, dim, ops8, False, False, tb)
        res8e = fref.four_time_8op(F(dm_1c), F(dm_2c), rho0, t1, F(prec_c), dt, dim, ops8, True, False, tb)
        res8l = fref.four_time_8op(F(dm_1c), F(dm_2c), rho0, t1, F(prec_c), dt, dim, ops8, False, True, tb)
        res4 = fref.four_time(F(dm_1c), F(dm_2c), rho0, t1, F(prec_c), dt, dim, ops8[0], ops8[1], ops8[2], ops8[3], tb)
        dyn = fref.dynamics_t1(F(dm_1c), F(dm_2c), rho0, t1, F(prec_c), dt, dim, tb)
        np.savez_compressed(os.path.join(HERE, f"fortran_timebin_d{dim}.npz"),
                            dm_1=dm_1c, dm_2=dm_2c, precalc=prec_c, rho_init=rho0, t1=t1, dt=dt, tb=tb,
                            ops8=np.stack(ops8), result8=np.asarray(res8), result8_early=np.asarray(res8e),
                            result8_late=np.asarray(res8l), result4=np.asarray(res4), dyn_t1=np.asarray(dyn))


def gen_pyref():
    sys.path.insert(0, REF_ROOT)
    from pyaceqd import pulses as P  # noqa: E402
    from pyaceqd import tools as T  # noqa: E402
    t = np.arange(-10.0, 40.0, 0.05)
    plist = {
        "chirped": P.ChirpedPulse(tau_0=3.0, e_start=0.3, alpha=10.0, t0=5.0, e0=1.0, phase=0.2),
        "chirped_polar": P.ChirpedPulse(tau_0=2.7, e_start=-1.0, alpha=40.0, t0=12.0, e0=5.3, polar_x=0.6),
        "gauss": P.Pulse(tau=2.0, e_start=0.5, w_gain=0.01, t0=3.0, e0=2.0, phase=0.1),
        "cw": P.CWLaser(e0=0.05, e_start=0.2),
        "smooth_rect": P.SmoothRectangle(tau=10.0, e_start=0.1, t0=15.0, e0=0.3, alpha_onoff=0.5),
        "asym": P.AsymmetricPulse(tau1=2.0, tau2=4.0, e_start=0.0, t0=7.0, e0=1.0),
    }
    arrs = {"t": t}
    for k, p in plist.items():
        arrs[f"{k}_total"] = np.asarray(p.get_total(t)) * np.ones_like(t)
        arrs[f"{k}_polar"] = np.array([p.polar_x, p.polar_y])
    train = P.PulseTrain(10.0, 3, P.ChirpedPulse(tau_0=3, e_start=-2.0, e0=1.0, t0=12), t_shift=1.0)
    arrs["train_total"] = train.get_total(t)
    fx, fy = train.get_total_xy(t)
    arrs["train_x"], arrs["train_y"] = fx, fy
    # integrals used by the non-uniform grid builders
    arrs["chirped_integral"] = plist["chirped"].get_integral(t)
    np.savez_compressed(os.path.join(HERE, "pyref_pulses.npz"), **arrs)

    # tools: time grids, dm composition, concurrence, dynamical-map time-localisation
    rng = np.random.default_rng(77)
    p1 = P.ChirpedPulse(tau_0=3, e_start=0, e0=1, t0=20)
    p2 = P.ChirpedPulse(tau_0=2, e_start=0, e0=1, t0=60)
    ct = T.construct_t(0, 100, 0.1, 1.0, None, p1, p2)
    ct_exp = T.construct_t(0, 400, 0.1, 2.0, 0.05, p1, simple_exp=True)
    sg = T.simple_t_gaussian(0, 40, 200, 0.1, 1.0, p1)
    outs = [np.arange(5.0)] + [rng.normal(size=5) + 1j * rng.normal(size=5) for _ in range(10)]
    tdm, rdm = T.compose_dm(outs, dim=4)
    rho4 = np.stack([rand_rho(4, rng) for _ in range(3)])
    conc = np.array([T.concurrence(r) for r in rho4])
    maps = rand_lindblad_maps(12, 2, 0.1, rng)
    dm_cum = np.empty_like(maps)
    acc = np.eye(4, dtype=complex)
    for i in range(12):
        acc = maps[i] @ acc
        dm_cum[i] = acc
    times = np.round(np.arange(13) * 0.1, 6)
    tl = T.calc_tl_dynmap_pseudo(dm_cum, times)
    ops_dm = {f"ops_dm_{k}": np.array(T.output_ops_dm(v)) for k, v in
              {"2": 2, "6": 6, "21": [2, 1], "22": [2, 2], "222": [2, 2, 2]}.items()}
    np.savez_compressed(os.path.join(HERE, "pyref_tools.npz"), construct_t=ct, construct_t_exp=ct_exp,
                        simple_t_gaussian=sg, compose_in=np.array(outs, dtype=complex), compose_t=tdm,
                        compose_rho=rdm, conc_rho=rho4, concurrence=conc, dm_cum=dm_cum, tl_times=times,
                        tl_maps=tl, **ops_dm)


def gen_polent():
    """pol_entanglement.G2 bookkeeping: the REFERENCE class (pyaceqd/pol_entanglement/G2.py) driven by the
    deterministic tests/fake_system.py model instead of ACE; our class runs on the same model in
    tests/test_callers_golden.py."""
    import tempfile
    import warnings
    warnings.simplefilter("ignore")
    sys.path.insert(0, REF_ROOT)
    from pyaceqd.pol_entanglement.G2 import PolarizatzionEntanglement as RefPE  # noqa: E402
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system  # noqa: E402
    tmp = tempfile.mkdtemp() + "/"
    p1 = ChirpedPulse(tau_0=1.0, e_start=1.0, alpha=0, e0=2.0, t0=5)
    opts = {"gamma_e": 1 / 100, "temp_dir": tmp, "lindblad": True}
    ops = ("|0><1|_4", "|0><2|_4", "|1><0|_4", "|2><0|_4")
    out = {}
    for tag, kw in {"ct": dict(dt=0.1, tend=14.0, dt_small=0.1), "reg": dict(dt=0.1, tend=6.0, dt_small=0.3,
                                                                             regular_grid=True)}.items():
        pe = RefPE(fake_system, *ops, p1, options=opts, **kw)
        out[f"{tag}_t1"] = pe.t1
        t1, t2, g, gi, full = pe.G2_reuse(pe.axdag, [pe.axdag + " * " + pe.ax, pe.aydag + " * " + pe.ay], pe.ax,
                                          return_full_G2=True)
        out.update({f"{tag}_reuse_t2": t2, f"{tag}_reuse_g": g, f"{tag}_reuse_int": gi, f"{tag}_reuse_full": full})
        _, g2, g2i = pe.G2(pe.axdag, pe.aydag, pe.ay, pe.ax)
        out.update({f"{tag}_g2": g2, f"{tag}_g2_int": np.array(g2i)})
        c, rho = pe.calc_densitymatrix_reuse(return_rho=True)
        out.update({f"{tag}_dm_reuse_c": np.array(c), f"{tag}_dm_reuse_rho": rho})
        out[f"{tag}_dm_c"] = np.array(pe.calc_densitymatrix(), dtype=complex)
        _, tt2, G1 = pe.G1(pe.ax, pe.axdag)
        out.update({f"{tag}_g1_t2": tt2, f"{tag}_g1": G1})
        fr, sp, sps = pe.get_spectrum(pe.ax, pe.axdag)
        out.update({f"{tag}_spec_f": fr, f"{tag}_spec": sp, f"{tag}_spectra0": sps[0]})
        for mode in ("t", "tau"):
            r = pe.calc_timedependent_rho(mode=mode, add_norm=0.05, skip=1, return_G2=True)
            for name, v in zip(("t", "c_t", "rho", "norm", "rho_int", "c_int", "G2_t"), r):
                out[f"{tag}_tdr_{mode}_{name}"] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, "pyref_polent.npz"), **out)


def _ref_with_fortran_module():
    """import path for reference modules that pull in the ACE-backed driver: pyaceqd/two_time/purity.py imports
    `tls` and two correlation functions at module level (purity.py:13-14) that the golden scenarios never call; their
    modules need the absent ACEutils library (general_system.py:14). Those two import targets are replaced by
    placeholders that raise if called, so nothing of ACE is imitated; the model is tests/fake_system.py. The f2py
    module `pyaceqd.two_time.propagate_tau_module` is provided by the reference's OWN Fortran compiled from
    propagate_tau.f90 (oracle/fref.py), i.e. the real reference arithmetic."""
    import types
    sys.path.insert(0, REF_ROOT)

    def _never(*a, **k):
        raise RuntimeError("not available offline (needs ACE)")
    for mod, names in {"pyaceqd.two_level_system.tls": ["tls"],
                       "pyaceqd.two_time.correlations": ["tl_two_op_two_time", "tl_three_op_two_time"]}.items():
        m = types.ModuleType(mod)
        for n in names:
            setattr(m, n, _never)
        sys.modules[mod] = m
    ptm = types.ModuleType("pyaceqd.two_time.propagate_tau_module")
    for name in ("propagate_tau", "calc_onetime_parallel", "calc_onetime_parallel_block", "calc_twotime_phonon_block"):
        setattr(ptm, name, getattr(fref, name))
    sys.modules["pyaceqd.two_time.propagate_tau_module"] = ptm


def _ref_correlations():
    """Import the reference's own pyaceqd/two_time/correlations.py. Its module-level import chain (correlations.py:6
    -> two_level_system/tls.py -> general_system.py:14) reaches the absent ACEutils pybind module; an empty placeholder
    (every imported name None, nothing callable: SURVEY.md §4.3) satisfies that import. The model callables passed to
    the reference functions are tests/fake_system.py or our own lowering on the CPU oracle (below), and
    `propagate_tau_module` is the reference's OWN Fortran (oracle/fref.py)."""
    import types
    sys.path.insert(0, REF_ROOT)
    for mod in ("pyaceqd.two_time.correlations", "pyaceqd.two_level_system.tls"):
        if mod in sys.modules and getattr(sys.modules[mod], "__file__", None) is None:
            del sys.modules[mod]  # placeholders left by _ref_with_fortran_module
    if "ACEutils" not in sys.modules:
        ace = types.ModuleType("ACEutils")
        for n in ("Parameters", "FreePropagator", "ProcessTensors", "InitialState", "OutputPrinter", "TimeGrid",
                  "Simulation", "read_outfile", "DynamicalMap"):
            setattr(ace, n, None)
        sys.modules["ACEutils"] = ace
    ptm = types.ModuleType("pyaceqd.two_time.propagate_tau_module")
    for name in ("propagate_tau", "calc_onetime_parallel", "calc_onetime_parallel_block", "calc_twotime_phonon_block"):
        setattr(ptm, name, getattr(fref, name))
    sys.modules["pyaceqd.two_time.propagate_tau_module"] = ptm
    import pyaceqd.two_time as pkg  # noqa: E402
    pkg.propagate_tau_module = ptm
    from pyaceqd.two_time import correlations  # noqa: E402
    return correlations


def gen_correlations():
    """two_time/correlations.py: the REFERENCE one-/two-time drivers (`_ops_one_time`, `_ops_two_time` and the four
    public wrappers, the time-local-map `tl_two_op_two_time` / `tl_three_op_two_time` in all three branches
    use_dm x fortran_only) on the deterministic tests/fake_system.py models; ours run the same calls in
    tests/test_callers_golden.py (CPU) and tests/test_gpu_parity.py (map-chain sweeps on the GPU)."""
    import io
    import contextlib
    import warnings
    warnings.simplefilter("ignore")
    R = _ref_correlations()
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system, fake_system_dm  # noqa: E402
    p = ChirpedPulse(tau_0=1.0, e_start=0, e0=1.5, t0=2)
    opts = lambda **k: dict({"lindblad": True, "phonons": False}, **k)  # noqa: E731
    t_axis = np.round(np.arange(7) * 0.3, 6)
    out = {"t_axis": t_axis}
    quiet = contextlib.redirect_stdout(io.StringIO())
    with quiet, contextlib.redirect_stderr(io.StringIO()):
        tau, G = R.two_op_one_time(fake_system, p, opA="|1><0|_2", opB="|0><1|_2", t0=-2, t_MTO=1.0, tend=4, dt=0.1,
                                   options=opts())
        out.update(ot2_tau=tau, ot2_G=G)
        tau, G = R.three_op_one_time(fake_system, p, t0=-2, t_MTO=1.0, tend=4, dt=0.1, options=opts())
        out.update(ot3_tau=tau, ot3_G=G)
        for tag, fn, kw in (("tt2", R.two_op_two_time, {}),
                            ("tt3", R.three_op_two_time, {}),
                            ("tt3s", R.three_op_two_time, {"t_start": -1.0}),
                            ("tt5", R.five_op_two_time, {"t_start": -1.0})):
            t1, t2, G = fn(fake_system, t_axis, p, tau_max=2.0, dt=0.1, options=opts(), workers=2, **kw)
            out.update({f"{tag}_t1": t1, f"{tag}_t2": t2, f"{tag}_G": G})
        rho2 = np.array([[0.8, 0.1 - 0.05j], [0.1 + 0.05j, 0.2]], dtype=complex)
        for tag, fn, kw in (("tl2", R.tl_two_op_two_time, {}),
                            ("tl3", R.tl_three_op_two_time, {"opC": "|0><1|_2"})):
            for use_dm, fo in ((False, False), (True, False), (True, True)):
                t1, t2, G = fn(fake_system_dm, t_axis, p, t_mem=1.0, tau_max=50.0, dt=0.1, rho0=rho2, opB="|0><0|_2",
                               options=opts(), use_dm=use_dm, fortran_only=fo, **kw)
                out[f"{tag}_dm{int(use_dm)}_f{int(fo)}_G"] = G
                out[f"{tag}_t2"] = t2
        # a non-hermitian-pair operator set on a 4-level fake model (the fortran_only view differs from the
        # row-major one there: both are pinned)
        rho4 = np.diag([0.5, 0.2, 0.2, 0.1]).astype(complex)
        rho4[0, 3] = rho4[3, 0] = 0.05
        for use_dm, fo in ((False, False), (True, False), (True, True)):
            t1, t2, G = R.tl_three_op_two_time(fake_system_dm, t_axis, p, t_mem=1.0, opA="|1><0|_4", opB="|2><1|_4",
                                               opC="|3><1|_4", tau_max=1.5, dt=0.1, rho0=rho4,
                                               options=opts(fake_dim=4), use_dm=use_dm, fortran_only=fo)
            out[f"tl3d4_dm{int(use_dm)}_f{int(fo)}_G"] = G
    np.savez_compressed(os.path.join(HERE, "pyref_correlations.npz"), **out)


def gen_correlations_phonons():
    """The rest of two_time/correlations.py: the REFERENCE get_spectrum (:322-380) on an analytic G1 (two damped
    lines plus an offset) and the two phonon dynamical-map functions tl_three_op_two_time_phonons (:866-1011) and
    tl_threeoptwotime_phonons_dm (:1013-1186) on tests/fake_system.py's calc_dynmap model (dim 2: their debugging
    code is written for 2x2, needs >= 10 t points and t_axis[-1] + tau_max >= 49.9 ps). They save figures to the relative path pyaceqd/tests/, so
    they run inside a scratch directory that has one."""
    import io
    import contextlib
    import tempfile
    import warnings
    warnings.simplefilter("ignore")
    R = _ref_correlations()
    import matplotlib
    matplotlib.use("Agg")
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system_dm  # noqa: E402
    tau = np.round(0.05 * np.arange(801), 6)
    g1 = (0.7 * np.exp(-0.3 * tau - 1j * 1.1 * tau) + 0.3 * np.exp(-0.8 * tau + 1j * 0.4 * tau)
          + 0.01 * (1 + 0.5j))
    s, om = R.get_spectrum(g1, tau)
    out = {"sp_g1": g1, "sp_tau": tau, "sp_s": s, "sp_omega": om}
    p = ChirpedPulse(tau_0=1.0, e_start=0, e0=1.5, t0=2)
    rho2 = np.array([[0.8, 0.1 - 0.05j], [0.1 + 0.05j, 0.2]], dtype=complex)
    t_axis = np.round(np.arange(12) * 0.2, 6)
    out["ph_t_axis"] = t_axis
    here = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "pyaceqd", "tests"))
        os.chdir(d)
        try:
            with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
                for tag, fn in (("ph", R.tl_three_op_two_time_phonons), ("phdm", R.tl_threeoptwotime_phonons_dm)):
                    _, tau2, G = fn(fake_system_dm, t_axis, p, t_mem=1.0, tau_max=50.0, dt=0.1, rho0=rho2, opB="|0><0|_2",
                                    options={"lindblad": True, "phonons": True,
                                             "output_ops": ["|0><0|_2", "|1><1|_2"]})
                    out[f"{tag}_tau"] = tau2
                    out[f"{tag}_G"] = G
        finally:
            os.chdir(here)
    np.savez_compressed(os.path.join(HERE, "pyref_correlations_phonons.npz"), **out)


def gen_twotime_anchor():
    """Reference-anchored two-time semantics of the PT path: exact no-phonon dynamical maps of a
    driven, decaying biexciton (our lowering of `biexciton`, propagated by the CPU oracle: dm[i] = E(t_{i+1}, 0)) are
    fed to the REFERENCE tl_three_op_two_time / tl_two_op_two_time (use_dm=True; time-localised by the reference's
    calc_tl_dynmap_pseudo, swept by the reference's own Fortran or its row-major Python path). The GPU test runs our
    trajectory sweep `three_op_two_time` / `two_op_two_time` (MTOs at t1 inside the PT kernel) on the same model and
    must reproduce these G within 1e-10. Both sides use the driver's default drive, pulse_sampling="ace_file" (the
    reference's %.8f pulse files on np.arange(t_start, t_end, dt); regenerated in round 4 when that became the
    default)."""
    import io
    import contextlib
    import warnings
    warnings.simplefilter("ignore")
    R = _ref_correlations()
    from oracle import oracle
    import pyaceqd_amd._lib as L
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.pulses import ChirpedPulse
    L.context = lambda device=None: None  # noqa: E731  (no device in the build container)
    gs.propagate = lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None: oracle.propagate(  # noqa: E731
        system, grid, rho0, out_ops, traj, pt=pt, nthreads=8)
    from pyaceqd_amd.engine import tables_from_outputs
    gs.propagate_table = lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None: tables_from_outputs(  # noqa
        gs.propagate(system, grid, rho0, out_ops, traj, pt=pt), traj, grid)
    p = ChirpedPulse(tau_0=1.0, e_start=-2.0, e0=1.3, t0=1.5, polar_x=0.8)
    t_axis = np.round(np.arange(8) * 0.5, 6)
    rho0 = np.zeros((4, 4), dtype=complex)
    rho0[0, 0] = 1.0
    opts = lambda: {"lindblad": True, "phonons": False, "delta_b": 4.0, "delta_xy": 0.03}  # noqa: E731
    out = {"t_axis": t_axis, "tau_max": 4.0, "dt": 0.1}
    with contextlib.redirect_stdout(io.StringIO()):
        for fo in (True, False):
            _, tau, G = R.tl_three_op_two_time(biexciton, t_axis, p, t_mem=0.5, opA="|3><1|_4", opB="|1><1|_4",
                                               opC="|1><3|_4", tau_max=4.0, dt=0.1, rho0=rho0, options=opts(),
                                               use_dm=True, fortran_only=fo)
            out[f"g2_f{int(fo)}"] = G
        _, tau, G = R.tl_two_op_two_time(biexciton, t_axis, p, t_mem=0.5, opA="|1><0|_4", opB="|0><1|_4",
                                         tau_max=4.0, dt=0.1, rho0=rho0, options=opts(), use_dm=True,
                                         fortran_only=False)
        out["g1_f0"] = G
    out["tau"] = tau
    np.savez_compressed(os.path.join(HERE, "pyref_twotime_anchor.npz"), **out)


def gen_params():
    """the ACE param text (and %.8f pulse files) the REFERENCE model functions write, captured with
    prepare_only=True (general_system.py:292-296; its module imports with the empty ACEutils placeholder of
    _ref_correlations). Temp-file paths are replaced by tokens. tests/test_params_golden.py lowers the same calls
    through our driver and checks every line's semantics (H0, Lindblad terms, pulse couplings and samples, initial
    state, outputs, multi-time operators)."""
    import io
    import json
    import contextlib
    import tempfile
    import warnings
    warnings.simplefilter("ignore")
    _ref_correlations()
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from pyaceqd.two_level_system.tls import tls  # noqa: E402
    from pyaceqd.four_level_system.linear import biexciton  # noqa: E402
    from pyaceqd.six_level_system.linear import sixls_linear  # noqa: E402
    p1 = ChirpedPulse(tau_0=1.0, e_start=0.2, e0=1.3, t0=2.0, alpha=5.0, phase=0.3)
    p2 = ChirpedPulse(tau_0=0.8, e_start=-1.0, e0=0.7, t0=3.0, polar_x=0.6)
    mto = [{"operator": "|0><1|_2", "applyFrom": "_left", "applyBefore": "false", "time": 1.5},
           {"operator": "|1><0|_2", "applyFrom": "_right", "time": 1.5},
           {"operator": "|1><1|_2", "applyFrom": "", "applyBefore": "true", "time": 2.0}]
    cases = {
        "tls": (tls, dict(dt=0.1, lindblad=True, multitime_op=mto, gamma_e=0.02)),
        "tls_dephasing": (tls, dict(dt=0.05, lindblad=True, dephasing=0.01, e_x=0.3)),
        "biexciton": (biexciton, dict(dt=0.1, lindblad=True, delta_xy=0.1, delta_b=3.0, gamma_b=0.03)),
        "sixls": (sixls_linear, dict(dt=0.1, bx=1.5, bz=0.5, lindblad=True)),
    }
    out = {}
    for name, (fn, kw) in cases.items():
        tmp = tempfile.mkdtemp() + "/"
        with contextlib.redirect_stdout(io.StringIO()):
            fn(0, 4, p1, p2, temp_dir=tmp, prepare_only=True, suffix="g", **kw)
        files = sorted(os.listdir(tmp))
        params = [f for f in files if f.endswith(".param")]
        assert len(params) == 1, files
        text = open(tmp + params[0]).read()
        rec = {"kwargs": {k: v for k, v in kw.items()}, "pulse_files": {}}
        for f in files:
            if f.endswith(".dat"):
                tok = "<PULSE_Y>" if "_y_" in f else "<PULSE_X>"
                text = text.replace(tmp + f, tok)
                rec["pulse_files"][tok] = open(tmp + f).read()
        text = text.replace(tmp, "<TMP>/")
        rec["param"] = text
        out[name] = rec
    with open(os.path.join(HERE, "pyref_params.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_purity():
    """two_time/purity.py bookkeeping and time-local-map paths: the REFERENCE Purity / Indistinguishability classes
    driven by tests/fake_system.fake_system_dm (analytic outputs + synthetic dynamical maps), with the reference
    Fortran behind propagate_tau_module; ours runs the same model in tests/test_callers_golden.py (GPU sweeps in
    tests/test_gpu_parity.py)."""
    import tempfile
    import warnings
    warnings.simplefilter("ignore")
    _ref_with_fortran_module()
    from pyaceqd.two_time.purity import Purity, Indistinguishability  # noqa: E402
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system_dm  # noqa: E402
    tmp = tempfile.mkdtemp() + "/"
    p = ChirpedPulse(tau_0=1.5, e_start=0, e0=1, t0=6)
    kw = dict(dt=0.1, tb=20, dt_small=0.5, gaussian_t=12)
    out = {}
    pu = Purity(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options={"gamma_e": 0.01, "temp_dir": tmp}, **kw)
    out["pu_t1"] = pu.t1
    t1, t2, G = pu.G2(return_whole=True)
    out.update({"pu_g2_t2": t2, "pu_g2_whole": G})
    out["pu_g2"] = pu.G2()[1]
    out["pu_g2mod"] = pu.G2_modified("|1><1|_2")[1]
    out["pu_purity"] = np.array(pu.calc_purity())
    ind = Indistinguishability(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options={"gamma_e": 0.01, "temp_dir": tmp},
                               **kw)
    out["in_g1"] = ind.G1()[1]
    out["in_g0"] = ind.simple_propagation()[1]
    out["in_indist"] = np.array(ind.calc_indistinguishability())
    opts = {"gamma_e": 0.01, "temp_dir": tmp, "phonons": False}
    tl = Indistinguishability(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options=opts, dm=True, **kw)
    tl.get_tl()
    out.update({"tl_map": tl.tl_map, "tl_dms": tl.tl_dms})
    out["tl_g0"] = tl.simple_propagation_tl()[1]
    tt, rho = tl.calc_timedynamics_tl()
    out.update({"tl_dyn_t": tt, "tl_dyn_rho": rho, "tl_complete": tl.tl_complete})
    out["tl_g1"] = tl.G1_tl()[1]
    out["tl_g2"] = tl.G2_tl()[1]
    out["tl_indist"] = np.array(tl.calc_indistinguishability())
    opts = {"gamma_e": 0.01, "temp_dir": tmp, "phonons": True}
    ph = Indistinguishability(fake_system_dm, "|0><1|_2", "|1><0|_2", p, options=opts, dm=True, t_mem=2, **kw)
    out["ph_g0"] = ph.simple_propagation_tl_phonons()[1]
    tt, rho = ph.calc_timedynamics_tl_phonons()
    out.update({"ph_dyn_t": tt, "ph_dyn_rho": rho})
    out["ph_g1"] = ph.G1_tl_phonons()[1]
    out["ph_g2"] = ph.G2_tl_phonons()[1]
    np.savez_compressed(os.path.join(HERE, "pyref_purity.npz"), **out)


def gen_g1():
    """two_time/G1.py G1_general bookkeeping: the REFERENCE function on tests/fake_system.fake_system"""
    import warnings
    warnings.simplefilter("ignore")
    _ref_with_fortran_module()
    from pyaceqd.two_time.G1 import G1_general  # noqa: E402
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system  # noqa: E402
    p = ChirpedPulse(tau_0=1.0, e_start=0, e0=2, t0=4)
    mto = {"operator": "|0><1|_2", "applyFrom": "_left", "applyBefore": "false"}
    opts = {"phonons": False, "output_ops": ["|1><1|_2", "|1><0|_2"], "gamma_e": 0.01}
    out = {}
    for tag, kw in {"fine": dict(coarse_t=False), "coarse": dict(coarse_t=True, simple_exp=False)}.items():
        t, tau, G = G1_general(0, 12, 0, 6, 0.5, 0.1, p, p, system=fake_system, multitime_op=mto, **kw, **opts)
        out.update({f"{tag}_t": t, f"{tag}_tau": tau, f"{tag}_G": G})
    np.savez_compressed(os.path.join(HERE, "pyref_g1.npz"), **out)


def gen_twophoton():
    """timebin/twophoton_new.py: the REFERENCE TwoPhotonTimebinNew on tests/fake_system.fake_system_dm. Its compiled
    helper `pyaceqd.timebin.timebin_tl` is provided by the reference's own Fortran (four_time, four_time_8op via
    oracle/fref.py); the two `utils` module functions the class calls from Python (fast_propagate, propagate_tb,
    timebin_tl.f90:23-77, module procedures returning arrays, which a C binding cannot reach) are restated below in
    numpy from that source."""
    import tempfile
    import types
    import warnings
    warnings.simplefilter("ignore")
    _ref_with_fortran_module()

    def fast_propagate(rho, pre, n_steps, dimsquare=None, n_precalc=None):
        out, n, i = np.array(rho, dtype=complex), int(n_steps), 0
        while n > 0:
            if n & 1:
                out = pre[:, :, i] @ out
            n >>= 1
            i += 1
        return out

    def propagate_tb(t_start, t_stop, dt, rho, dm_tl, pre, n_precalc=None, dimsquare=None, n_dm=None):
        r6 = lambda x: np.rint(x * 1e6) / 1e6  # noqa: E731
        n_start, n_stop = int(r6(t_start) / dt), int(r6(t_stop) / dt)
        n_steps = n_stop - n_start
        steps = min(dm_tl.shape[2] - n_start, n_steps)
        out = np.array(rho, dtype=complex)
        while steps > 0:
            out = dm_tl[:, :, n_start] @ out
            n_steps -= 1
            n_start += 1
            steps -= 1
        return fast_propagate(out, pre, n_steps) if n_steps > 0 else out
    tb_mod = types.ModuleType("pyaceqd.timebin.timebin_tl")
    tb_mod.four_time = lambda dm_1, dm_2, rho_init, t1, precalc, dt, dim, o1, o2, o3, o4, tb: fref.four_time(
        dm_1, dm_2, rho_init, t1, precalc, dt, dim, o1, o2, o3, o4, tb)
    tb_mod.four_time_8op = lambda dm_1, dm_2, rho_init, t1, precalc, dt, dim, *rest: fref.four_time_8op(
        dm_1, dm_2, rho_init, t1, precalc, dt, dim, rest[:8], rest[8], rest[9], rest[10])
    tb_mod.utils = types.SimpleNamespace(fast_propagate=fast_propagate, propagate_tb=propagate_tb)
    sys.modules["pyaceqd.timebin.timebin_tl"] = tb_mod
    import pyaceqd.timebin as pkg  # noqa: E402
    pkg.timebin_tl = tb_mod
    from pyaceqd.timebin.twophoton_new import TwoPhotonTimebinNew  # noqa: E402
    from pyaceqd.pulses import ChirpedPulse  # noqa: E402
    from tests.fake_system import fake_system_dm  # noqa: E402
    tmp = tempfile.mkdtemp() + "/"
    ps = [ChirpedPulse(tau_0=1.0, e_start=0, e0=1, t0=3), ChirpedPulse(tau_0=1.0, e_start=0, e0=1, t0=15)]
    ops = ("|0><1|_4", "|1><0|_4", "|1><3|_4", "|3><1|_4")
    opts = {"gamma_e": 0.05, "temp_dir": tmp, "fake_dim": 4}
    kw = dict(dt=0.1, dim=4, tb=12, dt_small=0.5, n_tbig=2, gaussian_t=6)
    out = {}
    tp = TwoPhotonTimebinNew(fake_system_dm, *ops, *ps, options=opts, **kw)
    out["t1"] = tp.t1
    c, rho = tp.calc_densitymatrix(reduced=False)
    out.update({"dm_c": np.array(c), "dm_rho": rho})
    r = tp.rho_ee_ee()
    out.update({"eeee_G": r[2], "eeee_table": r[6]})
    out["eell_table"] = tp.rho_ee_ll()[5]
    out["elll_G1"], out["elll_G2"] = tp.rho_el_ll()[3:5]
    tl = TwoPhotonTimebinNew(fake_system_dm, *ops, *ps, options=opts, **kw)
    c, rho, rhon = tl.calc_densitymatrix_tl(reduced=False)
    out.update({"tl_c": np.array(c), "tl_rho": rho})
    out["tl_eell_f"] = tl.eell_tl_f()[3]
    t, rho_t = tl.dynamics_tl()
    out.update({"tl_dyn_t": t, "tl_dyn_rho": rho_t})
    t, rho_t = tl.dynamics_tl_t1()
    out.update({"tl_dyn1_t": t, "tl_dyn1_rho": rho_t})
    ft = tl.four_time_tl(tp.sigma_bdag, tp.sigma_xdag, tp.sigma_b, tp.sigma_x)
    out.update({"tl_ft_G": ft[1], "tl_ft_table": ft[3]})
    np.savez_compressed(os.path.join(HERE, "pyref_twophoton.npz"), **out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["gen_" + name]()
        raise SystemExit(0)
    if not fref.available():
        raise SystemExit("build oracle/_ref first: make -C oracle ref")
    gen_fortran()
    gen_pyref()
    gen_correlations()
    gen_correlations_phonons()
    gen_twotime_anchor()
    gen_polent()
    gen_purity()
    gen_g1()
    gen_twophoton()
    tot = sum(os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE) if f.endswith(".npz"))
    print(f"golden fixtures written: {tot/1e6:.2f} MB")
