"""Operator grammar and model lowering pinned to the ACE param text the REFERENCE writes.

tests/golden/pyref_params.json holds the param files (and %.8f pulse files) of the reference's own `tls`,
`biexciton` and `sixls_linear`, captured with prepare_only=True (tests/golden/make_golden.py gen_params). Our model
functions are called with the same arguments; instead of running, the lowered engine inputs (System, Grid, rho0,
output operators, trajectories) are captured and every param line is checked against them:
  initial { s }               -> rho0 = s
  add_Hamiltonian { s }       -> H0 = sum of the s
  add_Lindblad r { s }        -> Lindblad term (r, s), in order
  add_Pulse file F { s }      -> pulse channel with coupling s (here -0.5*pi*hbar*(op)) and samples = file F at every
                                 dt (within the file's %.8f rounding)
  apply_Operator<side> t {s} b -> MTO at step round((t - ta)/dt), side, applyBefore b, operator s
  add_Output { s }            -> output operator s
Strings are evaluated with our grammar on both sides, so what this pins is that our model functions write the same
operator content, rates and couplings as the reference, and that the driver maps every line onto the engine as the
param file states it.
"""
import json
import os
import re

import numpy as np

from pyaceqd_amd.engine import tables_from_outputs
import pytest

from pyaceqd_amd import opgrammar
from pyaceqd_amd.pulses import ChirpedPulse


@pytest.fixture(scope="module")
def params(golden_dir):
    with open(os.path.join(golden_dir, "pyref_params.json")) as f:
        return json.load(f)


def _capture(monkeypatch):
    import pyaceqd_amd._lib as L
    from pyaceqd_amd.general_system import general_system as gs
    got = {}

    def prop(system, grid, rho0, out_ops, traj, pt=None, ctx=None):
        got.update(system=system, grid=grid, rho0=rho0, out_ops=out_ops, traj=traj)
        return [np.zeros((int(e - b + 1), len(out_ops)), dtype=complex) for b, e in zip(traj.out_begin, traj.out_end)]
    monkeypatch.setattr(L, "context", lambda device=None: None)
    monkeypatch.setattr(gs, "propagate", prop)
    monkeypatch.setattr(gs, "propagate_table", lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None:
                        tables_from_outputs(prop(system, grid, rho0, out_ops, traj, pt, ctx), traj, grid))
    return got


def _model(name):
    if name.startswith("tls"):
        from pyaceqd_amd.two_level_system.tls import tls
        return tls
    if name == "biexciton":
        from pyaceqd_amd.four_level_system.linear import biexciton
        return biexciton
    from pyaceqd_amd.six_level_system.linear import sixls_linear
    return sixls_linear


def _parse(text):
    lines = [ln.strip() for ln in text.splitlines() if ln.strip()]
    br = lambda ln: ln[ln.index("{") + 1: ln.rindex("}")].strip()  # noqa: E731
    rec = {"ham": [], "lind": [], "pulse": [], "mto": [], "out": []}
    for ln in lines:
        key = ln.split()[0]
        if key in ("dt", "ta", "te"):
            rec[key] = float(ln.split()[1])
        elif key == "initial":
            rec["initial"] = br(ln)
        elif key == "add_Hamiltonian":
            rec["ham"].append(br(ln))
        elif key == "add_Lindblad":
            rec["lind"].append((float(ln.split()[1]), br(ln)))
        elif key == "add_Pulse":
            rec["pulse"].append((ln.split()[2], br(ln)))
        elif key.startswith("apply_Operator"):
            m = re.match(r"apply_Operator(\S*)\s+(\S+)\s+\{(.*)\}\s+(\S+)", ln)
            rec["mto"].append((m.group(1), float(m.group(2)), m.group(3).strip(), m.group(4) == "true"))
        elif key == "add_Output":
            rec["out"].append(br(ln))
    return rec


@pytest.mark.parametrize("name", ["tls", "tls_dephasing", "biexciton", "sixls"])
def test_model_lowering_matches_reference_param_file(params, name, monkeypatch):
    g = params[name]
    rec = _parse(g["param"])
    kw = dict(g["kwargs"])
    p1 = ChirpedPulse(tau_0=1.0, e_start=0.2, e0=1.3, t0=2.0, alpha=5.0, phase=0.3)
    p2 = ChirpedPulse(tau_0=0.8, e_start=-1.0, e0=0.7, t0=3.0, polar_x=0.6)
    got = _capture(monkeypatch)
    _model(name)(0, 4, p1, p2, suffix="g", **kw)
    sysd, grid = got["system"], got["grid"]
    N = sysd.dim
    M = lambda s: opgrammar.to_matrix(s, N)  # noqa: E731
    assert grid.ta == rec["ta"] and grid.dt == rec["dt"] and grid.ta + grid.n_steps * grid.dt == pytest.approx(rec["te"])
    np.testing.assert_allclose(np.asarray(got["rho0"]).reshape(N, N), M(rec["initial"]), atol=0)
    H = sum((M(s) for s in rec["ham"]), np.zeros((N, N), dtype=complex))
    np.testing.assert_allclose(sysd.H0, H, rtol=1e-15, atol=1e-15)
    assert len(sysd.lindblad) == len(rec["lind"])
    for (r, L), (rr, s) in zip(sysd.lindblad, rec["lind"]):
        assert r == rr
        np.testing.assert_allclose(L, M(s), atol=0)
    assert len(sysd.channels) == len(rec["pulse"])
    n = grid.n_steps
    ts_file = rec["ta"] + rec["dt"] * np.arange(n)
    for (X, f), (tok, s) in zip(sysd.channels, rec["pulse"]):
        np.testing.assert_allclose(X, M(s), rtol=1e-15, atol=1e-15)
        d = np.loadtxt(g["pulse_files"][tok].splitlines())
        np.testing.assert_allclose(d[:, 0], ts_file, atol=5e-9)
        k = np.rint((ts_file - sysd.sample_t0) / sysd.sample_dt).astype(int)
        np.testing.assert_allclose(sysd.sample_t0 + k * sysd.sample_dt, ts_file, atol=1e-12)
        fs = np.asarray(f)[k]
        assert np.max(np.abs(fs.real - d[:, 1])) <= 5.01e-9 and np.max(np.abs(fs.imag - d[:, 2])) <= 5.01e-9
    outs = got["out_ops"]
    assert len(outs) == len(rec["out"])
    for O, s in zip(outs, rec["out"]):
        np.testing.assert_allclose(O, M(s), atol=0)
    mtos = got["traj"].mtos
    assert len(mtos) == len(rec["mto"])
    kinds = {"": 0, "_left": 1, "_right": 2}
    for m, (side, t, s, before) in zip(mtos, rec["mto"]):
        assert m.step == int(round((t - rec["ta"]) / rec["dt"])) and m.kind == kinds[side] and m.before == before
        np.testing.assert_allclose(m.op, M(s), atol=0)


@pytest.mark.parametrize("name", ["tls", "biexciton", "sixls"])
def test_ace_file_pulse_sampling_reads_what_the_reference_writes(params, name, monkeypatch):
    """pulse_sampling="ace_file": the engine's channel samples ARE the %.8f pulse files the reference writes for
    ACE (general_system.py:55-71, 213), bit for bit, on the file's own grid (t_start, dt); between samples the
    engine interpolates linearly and holds past t_end - dt, as for an explicit pulse_file_x/_y"""
    g = params[name]
    rec = _parse(g["param"])
    kw = dict(g["kwargs"])
    p1 = ChirpedPulse(tau_0=1.0, e_start=0.2, e0=1.3, t0=2.0, alpha=5.0, phase=0.3)
    p2 = ChirpedPulse(tau_0=0.8, e_start=-1.0, e0=0.7, t0=3.0, polar_x=0.6)
    got = _capture(monkeypatch)
    _model(name)(0, 4, p1, p2, suffix="g", pulse_sampling="ace_file", **kw)
    sysd = got["system"]
    assert len(sysd.channels) == len(rec["pulse"])
    for (X, f), (tok, s) in zip(sysd.channels, rec["pulse"]):
        d = np.loadtxt(g["pulse_files"][tok].splitlines())
        assert len(f) == len(d)
        np.testing.assert_array_equal(np.asarray(f).real, d[:, 1])
        np.testing.assert_array_equal(np.asarray(f).imag, d[:, 2])
        assert sysd.sample_t0 == d[0, 0] and sysd.sample_dt == d[1, 0] - d[0, 0]
    with pytest.raises(ValueError, match="pulse_sampling"):
        _model(name)(0, 4, p1, suffix="g", pulse_sampling="files", **kw)


def test_single_projector_matches_reference_op_to_matrix():
    """tools.op_to_matrix (reference tools.py:260-304: |n><m|_d only) for every projector of d = 2..6"""
    from pyaceqd_amd.tools import op_to_matrix
    for d in range(2, 7):
        for a in range(d):
            for b in range(d):
                e = np.zeros((d, d), dtype=complex)
                e[a, b] = 1
                for s in (f"|{a}><{b}|_{d}", f"(|{a}><{b}|_{d})"):
                    np.testing.assert_array_equal(op_to_matrix(s), e)
