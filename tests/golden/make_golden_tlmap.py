"""Golden vectors for the time-local dynamical maps (tests/golden/pyref_tlmap.npz).

Run in the build container only (imports the reference from /root/reference):
    python tests/golden/make_golden_tlmap.py

Outputs are the REFERENCE's own calc_tl_dynmap_pseudo (pyaceqd/tools.py:446-484: numpy pinv with
rcond=1e-12) on synthetic cumulative maps: products of random drifting Lindblad maps for map sizes
n = N^2 = 16, 25 (odd: exercises the dummy column of the Jacobi tournament) and 36, and rank-deficient
maps (3 exactly-zero singular values, so the rcond cut-off decides) at n = 4 and 16.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF_ROOT, rand_lindblad_maps  # noqa: E402


def cumulative(maps):
    out = np.empty_like(maps)
    acc = np.eye(maps.shape[1], dtype=complex)
    for i in range(len(maps)):
        acc = maps[i] @ acc
        out[i] = acc
    return out


def main():
    sys.path.insert(0, REF_ROOT)
    from pyaceqd import tools as T
    rng = np.random.default_rng(4242)
    arrs = {}
    for name, dim, n_maps in (("d4", 4, 40), ("d5", 5, 24), ("d6", 6, 24)):
        dm = cumulative(rand_lindblad_maps(n_maps, dim, 0.1, rng))
        times = np.round(np.arange(n_maps + 1) * 0.1, 6)
        arrs[f"{name}_dm"] = dm
        arrs[f"{name}_times"] = times
        arrs[f"{name}_tl"] = T.calc_tl_dynmap_pseudo(dm, times)
    for name, dim, n_maps in (("rank2", 2, 10), ("rank4", 4, 12)):
        n = dim * dim
        dm = cumulative(rand_lindblad_maps(n_maps, dim, 0.1, rng))
        X = rng.normal(size=(n, n)) + 1j * rng.normal(size=(n, n))
        Q, _ = np.linalg.qr(X)
        P = Q @ np.diag([1.0] * (n - 3) + [0.0] * 3) @ Q.conj().T
        dm = np.stack([d @ P for d in dm])
        times = np.round(np.arange(n_maps + 1) * 0.1, 6)
        arrs[f"{name}_dm"] = dm
        arrs[f"{name}_times"] = times
        arrs[f"{name}_tl"] = T.calc_tl_dynmap_pseudo(dm, times)
    np.savez_compressed(os.path.join(HERE, "pyref_tlmap.npz"), **arrs)
    print({k: v.shape for k, v in arrs.items()})


if __name__ == "__main__":
    main()
