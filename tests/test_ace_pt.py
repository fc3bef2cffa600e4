"""ACE PT-file reader (pqd_ace_pt_shape / pqd_ace_pt_read, pyaceqd_amd/ace_pt.py).

ACE's layout is undocumented offline and no ACE-made file exists here, so what is tested is the stated assumption
ACE_PTB_V0 (csrc/ace_pt.cpp): files written in it read back exactly (bonds growing from 1 and zero-padded), the
driver picks them up by the reference's own detection (`<pt_file>_initial`, general_system.py:153-156) and every
other layout is refused with PQD_ERR_UNSUPPORTED naming the file. Host-only code: runs without a GPU. Parity with
real ACE files is unpinned."""
import os

import numpy as np
import pytest

from pyaceqd_amd import _lib, ace_pt, pt as ptmod


def _pt(N=4, chi=8, n_init=5, seed=3):
    boson = np.diag([0, 1, 1, 2.0])[:N, :N]
    p = ptmod.synthetic_pt(boson, chi=chi, n_init=n_init, n_rep=1, seed=seed, eps=0.2, structured=False,
                           dictionary=True)
    return p


def test_round_trip_full_bond(tmp_path):
    p = _pt()
    name = str(tmp_path / "bx.ptr")
    ace_pt.write_ace_pt(name, p)
    for suf in ("_initial", "_initial_0", "_repeated", "_repeated_0"):
        assert os.path.exists(name + suf)
    q = ace_pt.read_ace_pt(name, 4, dt=0.1)
    assert q.n_init == p.n_init and q.n_slices == p.n_slices and q.chi == p.chi
    np.testing.assert_array_equal(q.Q, p.Q)
    np.testing.assert_array_equal(q.closure, p.closure)
    np.testing.assert_array_equal(q.gmap, p.gmap)
    np.testing.assert_array_equal(q.bond0, p.bond0)       # e_0 on both sides
    np.testing.assert_array_equal(q.closure0, p.closure0)


def test_round_trip_growing_bonds_zero_padded(tmp_path):
    """a PT grown from bond 1 (ACE's construction): elements of sizes (1x2), (2x4), (4x8), (8x8)..., padded to 8"""
    p = _pt(chi=8, n_init=4)
    bonds = [1, 2, 4, 8, 8, 8]
    Q = np.zeros_like(p.Q)
    cl = np.zeros_like(p.closure)
    for s in range(p.n_slices):
        bl, br = bonds[s], bonds[s + 1] if s < p.n_slices - 1 else bonds[s]
        Q[s, :, :bl, :br] = p.Q[s, :, :bl, :br]
        cl[s, :br] = p.closure[s, :br]
    p.Q, p.closure = Q, cl
    name = str(tmp_path / "grow")
    ace_pt.write_ace_pt(name, p, bonds=bonds)
    assert os.path.getsize(name + "_initial_0") < 4 * (16 * 3 * 64 * 16)  # cut to the true bonds
    q = ace_pt.read_ace_pt(name, 4)
    assert q.chi == 8
    np.testing.assert_array_equal(q.Q, Q)
    np.testing.assert_array_equal(q.closure, cl)


def _write_bad(tmp_path, mutate):
    name = str(tmp_path / "bad")
    ace_pt.write_ace_pt(name, _pt())
    mutate(name)
    return name


@pytest.mark.parametrize("case,match", [
    ("magic", "ACE_PTB_V0"), ("tag", "PTE0"), ("truncated", "truncated"), ("count", "announces"),
    ("dim", "Liouville dimension"), ("dict", "dictionary entry")])
def test_other_layouts_are_refused(tmp_path, case, match):
    def mutate(name):
        if case == "magic":     # e.g. a real ACE header: not the assumed layout
            open(name + "_initial", "w").write("some other header\n")
        elif case == "tag":
            b = bytearray(open(name + "_repeated_0", "rb").read())
            b[:4] = b"XXXX"
            open(name + "_repeated_0", "wb").write(bytes(b))
        elif case == "truncated":
            b = open(name + "_initial_0", "rb").read()
            open(name + "_initial_0", "wb").write(b[: len(b) - 100])
        elif case == "count":
            open(name + "_initial", "w").write("ACE_PTB_V0\nelements 9\nblocks 1\n")
        elif case == "dict":
            b = bytearray(open(name + "_initial_0", "rb").read())
            b[12:16] = np.int32(77).tobytes()
            open(name + "_initial_0", "wb").write(bytes(b))
    name = _write_bad(tmp_path, mutate if case != "dim" else (lambda n: None))
    with pytest.raises(_lib.PQDError, match=match) as ei:
        ace_pt.read_ace_pt(name, 2 if case == "dim" else 4)
    assert "libpqd error 3" in str(ei.value)     # PQD_ERR_UNSUPPORTED


def test_missing_files_raise_value_error(tmp_path):
    name = str(tmp_path / "half")
    ace_pt.write_ace_pt(name, _pt())
    os.remove(name + "_repeated_0")
    with pytest.raises(ValueError, match="_repeated_0"):
        ace_pt.read_ace_pt(name, 4)


def test_driver_uses_ace_files_by_reference_detection(tmp_path, monkeypatch):
    """biexciton(..., phonons=True, pt_file=<name>) with <name>_initial present loads ACE's files"""
    from pyaceqd_amd.engine import tables_from_outputs
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.general_system import general_system as gs
    from pyaceqd_amd.pulses import ChirpedPulse
    p = _pt(chi=8, n_init=30)
    name = str(tmp_path / "bx.ptr")
    ace_pt.write_ace_pt(name, p)
    got = {}

    def prop(system, grid, rho0, out_ops, traj, pt=None, ctx=None):
        got["pt"] = pt
        return [np.zeros((int(e - b + 1), len(out_ops)), dtype=complex) for b, e in zip(traj.out_begin, traj.out_end)]
    monkeypatch.setattr(_lib, "context", lambda device=None: None)
    monkeypatch.setattr(gs, "propagate_table", lambda system, grid, rho0, out_ops, traj, pt=None, ctx=None:
                        tables_from_outputs(prop(system, grid, rho0, out_ops, traj, pt, ctx), traj, grid))
    biexciton(0, 5, ChirpedPulse(tau_0=1, e_start=-2, e0=1, t0=2), dt=0.1, phonons=True, pt_file=name)
    q = got["pt"]
    assert q is not None and q.n_init == 30
    np.testing.assert_array_equal(q.Q, p.Q)
