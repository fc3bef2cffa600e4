"""ACE operator-string evaluation for every string form the reference models write."""
import numpy as np
import pytest

from pyaceqd_amd import opgrammar as G
from pyaceqd_amd.constants import hbar
from pyaceqd_amd.four_level_system.linear import biexciton_ops
from pyaceqd_amd.six_level_system.linear import sixls_ops, mu_b, g_ex, g_hx, g_ez, g_hz


def kb(N, a, b):
    m = np.zeros((N, N), dtype=complex)
    m[a, b] = 1
    return m


def test_basic_forms():
    assert np.array_equal(G.evaluate("|1><0|_2"), kb(2, 1, 0))
    assert np.allclose(G.evaluate("-4*|3><3|_4"), -4 * kb(4, 3, 3))
    assert np.allclose(G.evaluate("1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4"), np.diag([0, 1, 1, 2]))
    assert np.allclose(G.evaluate("(|1><0|_2*|1><1|_2*|0><1|_2)"), 0 * kb(2, 1, 1))  # antibunched G2(tau=0)
    assert np.allclose(G.evaluate("(|1><0|_2*|0><0|_2*|0><1|_2)"), kb(2, 1, 1))
    assert np.allclose(G.evaluate("|0><0|_2-|1><1|_2"), np.diag([1, -1]))
    assert np.allclose(G.evaluate("1e-05*|1><1|_2"), 1e-5 * kb(2, 1, 1))
    assert np.allclose(G.evaluate("-0.0*|1><1|_4"), 0 * kb(4, 1, 1))
    assert np.allclose(G.evaluate("sqrt(2)*i*|0><1|_2"), np.sqrt(2) * 1j * kb(2, 0, 1))
    assert np.isclose(G.evaluate("-0.5*pi*hbar"), -0.5 * np.pi * hbar)
    assert np.allclose(G.evaluate("(-0.5*hbar*(|1><1|_2))"), -0.5 * hbar * kb(2, 1, 1))


def test_tensor_products_and_modes():
    a = G.evaluate("|0><0|_2 otimes Id_2 otimes Id_2")
    assert np.allclose(a, np.kron(kb(2, 0, 0), np.eye(4)))
    b = G.evaluate("0.5*(Id_2 otimes n_3) + 0.1*(|1><1|_2 otimes bdagger_3 + |1><1|_2 otimes b_3)")
    bb = np.diag(np.sqrt([1.0, 2.0]), 1)
    ref = 0.5 * np.kron(np.eye(2), np.diag([0, 1, 2])) + 0.1 * (np.kron(kb(2, 1, 1), bb.T) + np.kron(kb(2, 1, 1), bb))
    assert np.allclose(b, ref)


def test_model_strings():
    so, bo, lo, io, rf = biexciton_ops(delta_xy=0.1, delta_b=4, lindblad=True, rf=True)
    H = sum(G.to_matrix(s, 4) for s in so)
    assert np.allclose(H, np.diag([0, -0.05, 0.05, -4]))
    assert np.allclose(G.to_matrix(bo, 4), np.diag([0, 1, 1, 2]))
    assert np.allclose(G.to_matrix(io[0][0], 4), kb(4, 1, 0) + kb(4, 3, 1))
    so, bo, lo, io, rf = sixls_ops(bx=2.0, bz=1.0, lindblad=True)
    H = sum(G.to_matrix(s, 6) for s in so)
    assert np.allclose(H, H.conj().T)
    c13 = -0.5 * mu_b * 2.0 * (g_ex + g_hx)
    assert np.isclose(H[1, 3], c13) and np.isclose(H[3, 1], c13)
    c21 = -0.5 * mu_b * 1.0 * (g_ez - 3 * g_hz)
    assert np.isclose(H[2, 1], -1j * c21) and np.isclose(H[1, 2], 1j * c21)


@pytest.mark.parametrize("bad", ["|2><0|_2", "|0><1|_2 + |0><1|_3", "foo*|0><0|_2", "(|0><0|_2", "1 + |0><0|_2"])
def test_errors(bad):
    with pytest.raises(ValueError):
        G.evaluate(bad)
