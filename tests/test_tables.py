"""Host logic of the ACE-table path and of the G2_reuse integrals (CPU; no device).

* engine.split_table / table_offsets: the layout pqd_propagate_table writes (per trajectory (1 + n_out) rows of its
  window, back to back) against engine.tables_from_outputs, the host form of the same assembly;
* PolarizatzionEntanglement._reuse_integrals: the trapezoid as one dot per row with the interior weights against
  np.trapezoid per row (reference pol_entanglement/G2.py:484-505)."""
import numpy as np

from pyaceqd_amd import engine
from pyaceqd_amd.engine import Grid, Trajectories
from pyaceqd_amd.pol_entanglement.G2 import PolarizatzionEntanglement


def test_split_table_layout_matches_host_assembly():
    rng = np.random.default_rng(0)
    beg = np.array([0, 3, 7, 2, 9])
    end = np.array([5, 3, 12, 20, 9])
    tr = Trajectories(beg, end)
    n_out = 3
    grid = Grid(-1.25, 0.1, 20)
    outs = [rng.normal(size=(e - b + 1, n_out)) + 1j * rng.normal(size=(e - b + 1, n_out)) for b, e in zip(beg, end)]
    want = engine.tables_from_outputs(outs, tr, grid)
    off, L = engine.table_offsets(tr, n_out)
    assert list(L) == [e - b + 1 for b, e in zip(beg, end)]
    flat = np.concatenate([w.reshape(-1) for w in want])
    assert off[-1] == flat.size
    got = engine.split_table(flat, tr, n_out)
    for g, w, b in zip(got, want, beg):
        assert g.shape == w.shape and np.array_equal(g, w)
        assert np.array_equal(g[0].real, -1.25 + 0.1 * np.arange(b, b + g.shape[1]))


def test_reuse_integrals_match_trapezoid_per_row():
    rng = np.random.default_rng(1)
    pe = PolarizatzionEntanglement.__new__(PolarizatzionEntanglement)
    pe.dt, pe.tend = 0.1, 4.0
    n_tau = int(round(pe.tend / pe.dt))
    pe.t1 = np.array([0.0, 0.1, 0.7, 2.3, 3.9, 4.0])
    n_pairs = 2
    res = []
    for t1 in pe.t1:
        L = n_tau + 1 - int(t1 / pe.dt) + 3  # the reference slices the last rows; extra leading rows are ignored
        res.append(rng.normal(size=(1 + 2 * n_pairs, L)) + 1j * rng.normal(size=(1 + 2 * n_pairs, L)))
    t1, g, gi = pe._reuse_integrals(res, n_pairs, n_tau)
    t2 = np.linspace(0, pe.tend, n_tau + 1)
    for i, r in enumerate(res):
        n_t2 = n_tau - int(pe.t1[i] / pe.dt)
        rows = PolarizatzionEntanglement._g2_rows(r, n_pairs, n_t2)
        ref = np.trapezoid(rows, t2[: n_t2 + 1], axis=1)
        assert np.allclose(g[:, i], ref, rtol=1e-13, atol=1e-13)
    assert np.allclose(gi, np.trapezoid(g, pe.t1, axis=1), rtol=1e-13, atol=1e-13)
