"""ACE's PT files (`<pt_file>_initial`, `_initial_0`, `_repeated`, `_repeated_0`, detected as the
reference does, general_system.py:153-157, 194-197) read by pqd_ace_pt_shape / pqd_ace_pt_read (csrc/ace_pt.cpp) and
propagated on the HIP path through the driver. The files are written by this package under the stated ACE_PTB_V0
layout: no ACE-made file exists offline, so this pins the reader + driver + GPU chain, not ACE's
own format."""
import numpy as np
import pytest

from pyaceqd_amd import ace_pt, pt as ptmod

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chi,n_init", [(16, 30), (32, 12)])
def test_driver_propagates_ace_pt_files_on_the_gpu(tmp_path, chi, n_init):
    """biexciton(..., phonons=True, pt_file=<name>) with the four files present gives, bit for bit, the result of the
    same PT handed over as a ProcessTensor (explicit slices, then the repeated one), and the PT acts (differs from
    phonons=False)"""
    from pyaceqd_amd.four_level_system.linear import biexciton
    from pyaceqd_amd.pulses import ChirpedPulse
    p = ptmod.synthetic_pt(np.diag([0, 1, 1, 2.0]), chi=chi, n_init=n_init, n_rep=1, seed=chi + n_init, eps=0.2,
                           structured=False, dictionary=True)
    name = str(tmp_path / "bx.ptr")
    ace_pt.write_ace_pt(name, p)
    pulse = ChirpedPulse(tau_0=1, e_start=-2, e0=1, t0=2)
    via_files = biexciton(0, 5, pulse, dt=0.1, phonons=True, pt_file=name)
    direct = biexciton(0, 5, pulse, dt=0.1, phonons=True, pt_file=p)
    bare = biexciton(0, 5, pulse, dt=0.1, phonons=False)
    assert len(via_files) == len(direct)
    for a, b in zip(via_files, direct):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    assert max(np.max(np.abs(np.asarray(a) - np.asarray(b))) for a, b in zip(direct[1:], bare[1:])) > 1e-6
