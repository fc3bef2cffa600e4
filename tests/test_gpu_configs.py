"""The five BASELINE.json configurations, each run through the HIP path at the size the
configuration names, with the checks that size allows. GPU only.

  config 1  "two_level_system Rabi, no phonons, 1000 steps"      tls(0, 100, ChirpedPulse(tau_0=3, e_start=0, e0=1,
            t0=20), dt=0.1, lindblad=True) through the drop-in driver vs the same lowering on the CPU oracle, and the
            Rabi population against a direct Lindblad master-equation integration (scipy, independent of both)
  config 2  "two_level_system with phonon PT, bond-dim 32"        2,048-point pulse-area scan x 10,000 steps, chi=32,
            on the register-resident quad kernel (pt_quad.hip): vs the batched kernel (PQD_QUAD=0) to 1e-11, vs the
            oracle on three full-length trajectories, and a structured PT (bond channel 0 decoupled) == bare dynamics
            with the trace preserved to 1e-10 over every step
  config 3  "four_level_system biexciton cascade, bond-dim 64"    tests/test_gpu_parity.py::test_c3_full_size_invariants
            (10,000 steps, chi=64) and ::test_sweep_pt_split_full_c3_single_run; here the single run vs the oracle
  config 4  "two_time G2(t, tau) sweep, 256 tau-points"           256 t1 trajectories x 10,000 tau-steps, chi=64,
            biexciton (bench.build_workload): an unstructured PT vs the oracle on a 16-point sub-grid at full length,
            and the structured PT == bare dynamics over the whole grid; one rank's 32-point shard equals its block
            of the whole-grid run bit for bit (the shard each of 8 GPUs runs)
  config 5  "six_level_system + pol_entanglement tomography scan" densitymatrix_reuse_scan (three launches for the
            grid) at chi=64 with the class's t1 grid and its 6/8/6 output operators vs each point run on its own, and
            vs the oracle at reduced tend

The reference states no numbers for these (ACE is absent): every comparison is against the CPU
oracle (oracle/pqd_oracle.c), a second HIP kernel, or a property the physics fixes. Tolerances: 1e-11 relative
between two GPU kernels, 1e-10 against the oracle over 10,000 steps (summation-order differences of a few 1e-16 per
step), far below the north star's 1e-8."""
import os
import sys

import numpy as np
import pytest

from oracle import oracle
from pyaceqd_amd import engine, opgrammar, pt as ptmod
from pyaceqd_amd.engine import Trajectories
from tests.test_gpu_parity import _oracle_patch, cmp_lists, rel

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _subset(tr, ids):
    """trajectories `ids` of tr as a Trajectories of their own (MTOs and systems remapped)"""
    ids = [int(i) for i in ids]
    remap = {t: k for k, t in enumerate(ids)}
    mt = [type(m)(remap[m.traj], m.step, m.before, m.kind, m.op) for m in tr.mtos if m.traj in remap]
    sysidx = None if tr.system is None else np.asarray(tr.system)[ids]
    return Trajectories(np.asarray(tr.out_begin)[ids], np.asarray(tr.out_end)[ids], mt, system=sysidx)


def _configs():
    sys.path.insert(0, os.path.join(HERE, "scripts"))
    import bench_configs
    return bench_configs


# ------------------------------------------------------------------------------------------------ config 1
@pytest.mark.parametrize("sampling", ["ace_file", "exact"])
def test_config1_tls_rabi_1000_steps(monkeypatch, sampling):
    """tls(0, 100, ...) through the driver (default pulse_sampling = "ace_file": the drive ACE reads from the
    reference's %.8f pulse files) vs the oracle, and rho_11 vs a direct adaptive integration of the Lindblad equation
    driven by the SAME field: the piecewise-linear interpolant of the %.8f samples on np.arange(0, 100, dt), held past
    the last sample (general_system.py:55-71, 213), or the analytic pulse for pulse_sampling="exact"."""
    from scipy.integrate import solve_ivp
    from pyaceqd_amd.constants import hbar
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.general_system.general_system import _ace_file_samples, _sample_pulses
    p = ChirpedPulse(tau_0=3, e_start=0, e0=1, t0=20)
    a = tls(0, 100, p, dt=0.1, lindblad=True, pulse_sampling=sampling)
    assert a.shape == (5, 1001)
    assert np.max(np.abs(a[1] + a[2] - 1)) < 1e-12          # populations sum to one
    _oracle_patch(monkeypatch)
    b = tls(0, 100, p, dt=0.1, lindblad=True, pulse_sampling=sampling)
    assert np.max(np.abs(a - b)) < 1e-12
    # Lindblad master equation of the same model (tls.py:24-29 strings: H = -pi hbar/2 (f |1><0| + h.c.), decay
    # |0><1| at 1/100 per ps), integrated directly with an adaptive RK; the engine's symmetric Trotter steps at
    # dt = 0.1 differ by O(dt^2)
    g = 1 / 100
    s = np.array([[0, 1], [0, 0]], complex)      # |0><1|
    if sampling == "ace_file":
        tf, fx, _ = _ace_file_samples(np.arange(0, 100, 0.1), *_sample_pulses([p], np.arange(0, 100, 0.1)))
        field = lambda t: complex(np.interp(t, tf, fx.real) + 1j * np.interp(t, tf, fx.imag))  # noqa: E731
    else:
        field = lambda t: complex(p.get_total(np.array([t]))[0])  # noqa: E731

    def rhs(t, y):
        r = y.reshape(2, 2)
        f = field(t)
        X = -0.5 * np.pi * hbar * np.array([[0, 0], [1, 0]], complex)
        H = f * X + np.conj(f) * X.conj().T
        d = -1j / hbar * (H @ r - r @ H) + g * (s @ r @ s.conj().T - 0.5 * (s.conj().T @ s @ r + r @ s.conj().T @ s))
        return d.ravel()
    sol = solve_ivp(rhs, (0, 100), np.array([1, 0, 0, 0], complex), t_eval=[25.0, 40.0, 100.0], rtol=1e-11,
                    atol=1e-13, method="DOP853", max_step=0.05 if sampling == "ace_file" else np.inf)
    exc = sol.y[3].real        # rho_11 (measured: 0.95222, 0.82790, 0.45436; engine within 2.2e-7 ace_file, 6.7e-7 exact)
    assert np.max(np.abs(a[2][[250, 400, 1000]].real - exc)) < 1e-5
    assert exc[0] > 0.9                            # a pi pulse: the dot is inverted, then decays


def _exact_lindblad(H, lind, rho0, ops, ts):
    """<op>(t) = tr(op exp(L t) rho0) for a time-independent Lindbladian (row-major vec, scipy expm): the exact
    solution, independent of the oracle and of the engine's step structure"""
    import scipy.linalg as sla
    from pyaceqd_amd.constants import hbar
    N = H.shape[0]
    eye = np.eye(N)
    L = -1j / hbar * (np.kron(H, eye) - np.kron(eye, H.T))
    for Lk, g in lind:
        LdL = Lk.conj().T @ Lk
        L = L + g * (np.kron(Lk, Lk.conj()) - 0.5 * np.kron(LdL, eye) - 0.5 * np.kron(eye, LdL.T))
    rows = []
    for t in ts:
        r = (sla.expm(L * t) @ rho0.reshape(-1)).reshape(N, N)
        rows.append([np.trace(o @ r) for o in ops])
    return np.array(rows).T


@pytest.mark.parametrize("sampling", ["ace_file", "exact"])
def test_cw_drive_matches_exact_lindblad_solution(sampling):
    """No phonons and a constant (resonant CW) drive make the Lindbladian time independent, so the engine's symmetric
    Trotter steps must reproduce exp(L t) exactly: the HIP path (driver -> free propagators -> sweep -> output table)
    against scipy's matrix exponential at 1e-11 over 2,000 steps, two orders inside the north star's 1e-8 no-phonon
    tolerance, with neither the CPU oracle nor the engine's own lowering in the reference. TLS (tls.py strings) and the
    biexciton with both polarisation channels, fine-structure splitting and x-y coupling (linear.py strings, pinned
    to the reference's param text by test_params_golden.py). The ACE-file drive quantises the samples to %.8f, so the
    exact solution uses the quantised amplitudes (general_system.py:55-71)."""
    from pyaceqd_amd.constants import hbar
    from pyaceqd_amd.pulses import CWLaser
    from pyaceqd_amd.two_level_system.tls import tls
    from pyaceqd_amd.four_level_system.linear import biexciton, biexciton_ops
    q = (lambda v: float("%.8f" % v)) if sampling == "ace_file" else (lambda v: v)
    e0 = 0.3
    a = tls(0, 200, CWLaser(e0), dt=0.1, lindblad=True, pulse_sampling=sampling)
    assert a.shape == (5, 2001)
    X = -0.5 * np.pi * hbar * np.array([[0, 0], [1, 0]], complex)
    H = q(e0) * (X + X.conj().T)
    ops = [opgrammar.to_matrix(o, 2) for o in ["|0><0|_2", "|1><1|_2", "|0><1|_2", "|1><0|_2"]]
    idx = np.arange(0, 2001, 40)
    ref = _exact_lindblad(H, [(np.array([[0, 1], [0, 0]], complex), 1 / 100)], np.diag([1.0, 0]).astype(complex),
                          ops, a[0].real[idx])
    assert np.max(np.abs(a[1:, idx] - ref)) < 1e-11
    assert np.ptp(ref[1].real) > 0.5                   # Rabi oscillations, damped
    px = np.cos(0.3)
    so, _, lo, io, _ = biexciton_ops(lindblad=True, delta_xy=0.1, coupl_xy=0.02)
    b = biexciton(0, 200, CWLaser(0.5, polar_x=px), dt=0.1, lindblad=True, delta_xy=0.1, coupl_xy=0.02,
                  pulse_sampling=sampling)
    H = sum(opgrammar.to_matrix(o, 4) for o in so)
    for op, ch in io:
        f = q(0.5 * (px if ch == "x" else np.sqrt(1 - px ** 2)))
        Xc = -0.5 * np.pi * hbar * opgrammar.to_matrix(op, 4)
        H = H + f * (Xc + Xc.conj().T)
    lind = [(opgrammar.to_matrix(o, 4), g) for o, g in lo]
    ops = [opgrammar.to_matrix("|%d><%d|_4" % (k, k), 4) for k in range(4)]
    ref = _exact_lindblad(H, lind, np.diag([1.0, 0, 0, 0]).astype(complex), ops, b[0].real[idx])
    assert np.max(np.abs(b[1:, idx] - ref)) < 1e-11
    assert min(np.max(ref[k].real) for k in range(1, 4)) > 5e-3    # every level is reached (|3>: 0.008)


# ------------------------------------------------------------------------------------------------ config 2
def _c2(structured):
    bc = _configs()
    N, systems, grid, pt, rho0, ops, tr = bc.workload(**bc.CONFIGS["c2"])
    assert (N, len(systems), tr.n_traj, grid.n_steps, pt.chi) == (2, 2048, 2048, 10000, 32)
    if not structured:
        pt = ptmod.synthetic_pt(opgrammar.to_matrix("1.000*|1><1|_2", 2), chi=32, n_init=410, n_rep=1, seed=99,
                                eps=0.05, dt=0.1, structured=False)
    return systems, grid, pt, rho0, ops + [np.eye(2)], tr


def _plan_run(systems, grid, rho0, ops, tr, pt):
    plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    return plan.download(), plan.info()[0]


def test_config2_tls_chi32_full_scan_quad_vs_batched_and_oracle(monkeypatch):
    monkeypatch.setenv("PQD_SPLIT", "0")
    systems, grid, pt, rho0, ops, tr = _c2(structured=False)
    a, path = _plan_run(systems, grid, rho0, ops, tr, pt)
    assert path == "register-resident TLS quads"
    ids = [0, 1023, 2047]
    sub = _subset(tr, ids)
    ref = oracle.propagate([systems[i] for i in ids], grid, rho0, ops,
                           Trajectories(sub.out_begin, sub.out_end, sub.mtos, system=np.arange(3)), pt=pt, nthreads=8)
    cmp_lists([a[i] for i in ids], ref, 1e-10)
    monkeypatch.setenv("PQD_QUAD", "0")
    b, path = _plan_run(systems, grid, rho0, ops, tr, pt)
    assert path == "batched lock-step sweep"
    cmp_lists(a, b, 1e-11)


def test_config2_tls_chi32_full_scan_structured_pt_is_bare_dynamics(monkeypatch):
    monkeypatch.setenv("PQD_SPLIT", "0")
    systems, grid, pt, rho0, ops, tr = _c2(structured=True)
    a, path = _plan_run(systems, grid, rho0, ops, tr, pt)
    assert path == "register-resident TLS quads"
    b, _ = _plan_run(systems, grid, rho0, ops, tr, None)
    for x, y in zip(a, b):
        assert np.max(np.abs(x - y)) < 1e-10
        assert np.max(np.abs(x[:, -1] - 1)) < 1e-10           # trace preserved at every step
    assert max(float(np.max(np.abs(x[:, 0]))) for x in a) > 0.1   # the scan drives the dots


# ------------------------------------------------------------------------------------------------ config 3
def test_config3_biexciton_chi64_single_run_vs_oracle():
    """the reference's single-run case: one biexciton trajectory, chi = 64, 10,000 steps (split groups, §4.6)"""
    bc = _configs()
    N, sysd, grid, pt, rho0, ops, tr = bc.workload(**bc.CONFIGS["c3one"])
    pt = ptmod.synthetic_pt(opgrammar.to_matrix("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4", 4), chi=64, n_init=410,
                            n_rep=1, seed=5, eps=0.05, dt=0.1, structured=False)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert got[0].shape == (10001, 2)
    cmp_lists(got, oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=8), 1e-10)


# ------------------------------------------------------------------------------------------------ config 4
def _c4(structured):
    import bench
    sysd, grid, pt, rho0, ops, tr = bench.build_workload(256, 10000, 64, scan=1)
    if not structured:
        pt = ptmod.synthetic_pt(opgrammar.to_matrix("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4", 4), chi=64, n_init=410,
                                n_rep=1, seed=77, eps=0.05, dt=0.1, structured=False)
    assert tr.n_traj == 256 and int(tr.out_end[-1] - tr.out_begin[-1]) == 10000
    return sysd, grid, pt, rho0, ops, tr


def test_config4_g2_sweep_256_t1_full_length_vs_oracle_subgrid():
    sysd, grid, pt, rho0, ops, tr = _c4(structured=False)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert got[0].shape == (10001, 2)
    ids = np.arange(0, 256, 16)
    ref = oracle.propagate(sysd, grid, rho0, ops, _subset(tr, ids), pt=pt, nthreads=16)
    cmp_lists([got[i] for i in ids], ref, 1e-10)
    # G2(t1, 0) = <A B C>(t1) lives in output 1 at the first row; the sweep is not trivially zero
    assert max(abs(g[0, 1]) for g in got) > 0


def test_config4_g2_sweep_256_t1_structured_pt_is_bare_and_shards_are_exact():
    sysd, grid, pt, rho0, ops, tr = _c4(structured=True)
    a = engine.propagate(sysd, grid, rho0, ops, tr, pt=pt)
    b = engine.propagate(sysd, grid, rho0, ops, tr)
    for x, y in zip(a, b):
        assert np.max(np.abs(x - y)) < 1e-10
    # one GPU's shard of the 8-GPU split (32 t1 points per GPU) as a launch of its own
    from pyaceqd_amd import scan as scanmod
    import bench
    for rank in (0, 7):
        lo, hi = scanmod.shard_range(256, rank, 8)
        s2, g2, p2, r2, o2, t2 = bench.build_workload(hi - lo, 10000, 64, scan=1, t1_offset=lo)
        part = engine.propagate(s2, grid, r2, o2, t2, pt=pt)
        for k in range(hi - lo):
            assert np.array_equal(part[k], a[lo + k]) or rel(part[k], a[lo + k]) < 1e-13


def test_config4_generated_chi128_pt_full_length_vs_oracle_subgrid():
    """the workload the drop-in produces with phonons: the C4 shape (8 scan points x 256 t1 x
    10,000 tau steps, 2,048 trajectories) on a biexciton PT GENERATED on the GPU at dt = 0.1 with the reference's
    bath parameters (a_e 3 nm, 4 K, threshold 1e-10, bond cap 128; memory 4.1 ps here instead of 20.48 to keep the
    generation to seconds): chi = 128 and a 9-entry dictionary, so the sweep runs pt_sweep_kernel<16, 128, 4> with
    dictionary PT units. 16 trajectories spread over every scan point against the oracle at full length."""
    import bench
    from pyaceqd_amd import ptgen_gpu
    sysd, grid, _, rho0, ops, tr = bench.build_workload(256, 10000, 128, scan=8, make_pt=False)
    B = opgrammar.to_matrix("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4", 4)
    pt = ptgen_gpu.qd_phonon_pt_gpu(B, 0.1, t_mem=4.1, ae=3.0, temperature=4, threshold=1e-10)
    assert pt.chi == 128 and pt.D == 9 and pt.meta["K"] == 41
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    got = plan.download()
    assert len(got) == 2048 and got[0].shape == (10001, 2)
    ids = np.arange(0, 2048, 128) + np.arange(16) % 7
    ref = oracle.propagate(sysd, grid, rho0, ops, _subset(tr, ids), pt=pt, nthreads=16)
    cmp_lists([got[i] for i in ids], ref, 1e-10)
    assert max(abs(g[0, 1]) for g in got) > 0


# ------------------------------------------------------------------------------------------------ config 5
SX, SY = "|0><1|_6 + |1><5|_6", "|0><2|_6 + |2><5|_6"
SXD, SYD = "|1><0|_6 + |5><1|_6", "|2><0|_6 + |5><2|_6"


def _c5_insts(tend, tmp_path, e0s=(3.0, 5.5), bxs=(0.0, 2.0), t0=3.0, t0b=6.0, dt_small=None):
    from pyaceqd_amd.pol_entanglement.G2 import PolarizatzionEntanglement
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.six_level_system.linear import energies_linear, sixls_linear, sixls_ops
    E_X, _, _, _, E_B = energies_linear(delta_B=4)
    pt = ptmod.synthetic_pt(opgrammar.to_matrix(sixls_ops()[1], 6), chi=64, n_init=410, n_rep=1, seed=5, eps=0.05,
                            dt=0.1, dictionary=True, structured=False)
    insts, kws = [], []
    for e0 in e0s:
        for bx in bxs:
            p1 = ChirpedPulse(tau_0=2.7, e_start=E_X, alpha=40, e0=e0, t0=t0)
            p2 = ChirpedPulse(tau_0=2.7, e_start=E_B - E_X, alpha=40, e0=4.06, t0=t0b)
            opts = {"lindblad": True, "gamma_e": 1 / 100, "phonons": True, "pt_file": pt,
                    "temp_dir": str(tmp_path) + "/"}
            kw = dict(regular_grid=True, dt_small=dt_small) if dt_small else {}
            insts.append(PolarizatzionEntanglement(sixls_linear, SX, SY, SXD, SYD, p1, p2, dt=0.1, tend=tend,
                                                   options=opts, **kw))
            kws.append({"bx": bx})
    return insts, kws


def _c5_per_point(insts, kws):
    from functools import partial
    from pyaceqd_amd.six_level_system.linear import sixls_linear
    out = []
    for inst, kw in zip(insts, kws):
        inst.system = partial(sixls_linear, **kw)
        out.append(inst.calc_densitymatrix_reuse(return_rho=True))
    return out


def test_config5_tomography_scan_chi64_vs_per_point_runs(tmp_path):
    """chi = 64 dictionary PT, the class's own (non-regular) t1 grid, tend 180 ps, the chirped pulses (4 tau = 60 ps) inside
    [0, tend] as construct_t requires: 2 e0 x 2 bx points"""
    from pyaceqd_amd.pol_entanglement.G2 import densitymatrix_reuse_scan
    insts, kws = _c5_insts(180.0, tmp_path, t0=62.0, t0b=92.0)
    got = densitymatrix_reuse_scan(insts, kws, return_rho=True)
    assert len(insts[0].t1) > 100 and 0 <= min(insts[0].t1) and max(insts[0].t1) <= 180.0
    ref = _c5_per_point(*_c5_insts(180.0, tmp_path, t0=62.0, t0b=92.0))
    for (cg, rg), (cr, rr) in zip(got, ref):
        assert rg.shape == (4, 4)
        assert np.max(np.abs(rg - rr)) <= 1e-11 * np.max(np.abs(rr))
        assert abs(cg - cr) < 1e-9
    assert np.max(np.abs(got[0][1] - got[1][1])) > 1e-6 * np.max(np.abs(got[0][1]))   # bx matters


def test_config5_tomography_scan_chi64_vs_oracle(monkeypatch, tmp_path):
    from pyaceqd_amd.pol_entanglement.G2 import densitymatrix_reuse_scan
    insts, kws = _c5_insts(12.0, tmp_path, dt_small=1.0)
    got = densitymatrix_reuse_scan(insts, kws, return_rho=True)
    _oracle_patch(monkeypatch)
    ref = _c5_per_point(*_c5_insts(12.0, tmp_path, dt_small=1.0))
    for (cg, rg), (cr, rr) in zip(got, ref):
        assert np.max(np.abs(rg - rr)) <= 1e-10 * np.max(np.abs(rr))
        assert abs(cg - cr) < 1e-8


def test_config5_tomography_scan_chi64_180ps_vs_oracle_subsets(monkeypatch, tmp_path):
    """C5 at chi = 64 over the class's own (non-regular) t1 grid to tend 180 ps, as C4 is checked: every G2_reuse
    variant's launch (the whole 2 e0 x 2 bx grid in one multi-system launch, ~7,000 trajectories) is checked on 4 of
    its trajectories (first, one third, two thirds, last; different grid points) against the C oracle propagating
    the same trajectories. Tables are downloaded (PQD_SCAN_TRAPZ=0) so the per-trajectory outputs can be compared;
    the device-trapz path is compared with the table path in test_output_trapz_matches_host_integrals."""
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd.pol_entanglement.G2 import densitymatrix_reuse_scan
    monkeypatch.setenv("PQD_SCAN_TRAPZ", "0")
    real = gs.propagate_table
    checked = []

    def wrapped(system, grid, rho0, out_ops, traj, pt=None, ctx=None):
        res = real(system, grid, rho0, out_ops, traj, pt=pt, ctx=ctx)
        n = traj.n_traj
        ids = sorted({0, n // 3, (2 * n) // 3, n - 1})
        sub = _subset(traj, ids)
        ref = engine.tables_from_outputs(oracle.propagate(system, grid, rho0, out_ops, sub, pt=pt, nthreads=16),
                                         sub, grid)
        for k, i in enumerate(ids):
            assert np.array_equal(res[i][0], ref[k][0])      # the time rows
            checked.append((n, int(traj.out_end[i]), rel(res[i][1:], ref[k][1:])))
        return res
    monkeypatch.setattr(gs, "propagate_table", wrapped)
    insts, kws = _c5_insts(180.0, tmp_path, t0=62.0, t0b=92.0)
    got = densitymatrix_reuse_scan(insts, kws, return_rho=True)
    assert len(got) == 4 and len(insts[0].t1) > 100
    assert len(checked) == 12, checked                       # 3 variants x 4 trajectories
    assert all(n > 400 for n, _, _ in checked)               # each launch carries the whole grid
    assert max(e for _, e, _ in checked) >= 1700             # trajectories run to ~tend
    assert max(r for _, _, r in checked) < 1e-10, checked
