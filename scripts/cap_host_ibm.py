"""Host-generator check of what the bond cap costs at the tls phonon defaults (dt 0.1, a_e 5 nm, 4 K): generate a PT
with the host restatement (ptgen.py) at memory K, threshold thr and bond cap (0 = none), propagate an undriven dot on
the CPU oracle for 40 ps and compare the coherence with the closed-form independent-boson solution.
usage: python scripts/cap_host_ibm.py K thr cap   (logs of 65 1e-10 128 / 65 1e-10 0 / 65 1e-11 0: profiles/r06/chi256/)
"""
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from pyaceqd_amd import ptgen
from oracle import ptgen_oracle
from oracle import oracle
from pyaceqd_amd.engine import System, Grid, Trajectories
dt = 0.1
J = lambda w: ptgen.qd_phonon_J(w, ae=5.0)
K = int(sys.argv[1]); thr = float(sys.argv[2]); cap = int(sys.argv[3])
eta, delta = ptgen.eta_coefficients(J, 4.0, dt, K)
t0 = time.time()
pt = ptgen.build_gaussian_pt(np.diag([0.0, 1.0]), dt, eta, delta, threshold=thr, max_bond=cap)
print("K", K, "thr", thr, "cap", cap, "chi", pt.chi, "gen s", round(time.time() - t0, 1), pt.meta.get("truncation"), flush=True)
n = 400
out = oracle.propagate(System(dim=2, H0=np.zeros((2, 2))), Grid(0.0, dt, n), 0.5 * np.ones((2, 2), complex),
                       [np.array([[0, 1], [0, 0]], complex), np.eye(2)], Trajectories(np.array([0]), np.array([n])), pt=pt)[0]
t = dt * np.arange(n + 1)
ex = ptgen_oracle.ibm_coherence_exact(J, 4.0, t)
exd = ptgen_oracle.ibm_coherence_discrete(eta, delta, dt, n)
print("max rel err vs exact", np.max(np.abs(out[:, 0] - ex) / np.abs(ex)), "vs discrete", np.max(np.abs(out[:, 0] - exd) / np.abs(exd)), flush=True)
