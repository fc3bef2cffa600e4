"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement (oracle/pqd_oracle.c, oracle/mapchain_oracle.c) is the checker for the HIP
path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it. It consumes
the same engine dataclasses (pyaceqd_amd.engine.System/Grid/ProcessTensor/Trajectories) so a test
hands identical inputs to both sides.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("PQD_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")  # tests/test_asan.py: ASan build
_lib = None

P_C = C.POINTER(C.c_double)  # complex as interleaved doubles
P_I32 = C.POINTER(C.c_int32)
P_I64 = C.POINTER(C.c_int64)
P_F = C.POINTER(C.c_double)


class or_system(C.Structure):
    _fields_ = [("dim", C.c_int), ("hbar", C.c_double), ("H0", P_C), ("n_lind", C.c_int), ("lind_rates", P_F),
                ("lind_ops", P_C), ("n_chan", C.c_int), ("chan_ops", P_C), ("chan_samples", P_C),
                ("n_samples", C.c_int), ("sample_t0", C.c_double), ("sample_dt", C.c_double)]


class or_grid(C.Structure):
    _fields_ = [("ta", C.c_double), ("dt", C.c_double), ("n_steps", C.c_int), ("n_sub", C.c_int)]


class or_pt(C.Structure):
    _fields_ = [("chi", C.c_int), ("D", C.c_int), ("n_slices", C.c_int), ("Q", P_C), ("closure", P_C),
                ("closure0", P_C), ("bond0", P_C), ("gmap", P_I32), ("sched", P_I32)]


class or_traj(C.Structure):
    _fields_ = [("n_traj", C.c_int), ("out_begin", P_I32), ("out_end", P_I32), ("out_offset", P_I64),
                ("n_mto", C.c_int), ("mto_traj", P_I32), ("mto_step", P_I32), ("mto_before", P_I32),
                ("mto_kind", P_I32), ("mto_ops", P_C)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.or_propagate.restype = C.c_int
        _lib.or_propagate_blocked.restype = C.c_int
        _lib.or_free_propagators.restype = C.c_int
    return _lib


def _c(a):
    return np.ascontiguousarray(a, dtype=np.complex128)


def _p(a):
    return None if a is None else a.ctypes.data_as(P_C)


def _system(sysd, keep):
    N = sysd.dim
    s = or_system()
    keep.append(_c(sysd.H0))
    s.dim, s.hbar, s.H0 = N, sysd.hbar, _p(keep[-1])
    s.n_lind = len(sysd.lindblad)
    if sysd.lindblad:
        keep.append(np.ascontiguousarray([r for r, _ in sysd.lindblad], dtype=np.float64))
        s.lind_rates = keep[-1].ctypes.data_as(P_F)
        keep.append(_c(np.stack([o for _, o in sysd.lindblad])))
        s.lind_ops = _p(keep[-1])
    s.n_chan = len(sysd.channels)
    if sysd.channels:
        keep.append(_c(np.stack([x for x, _ in sysd.channels])))
        s.chan_ops = _p(keep[-1])
        keep.append(_c(np.stack([f for _, f in sysd.channels])))
        s.chan_samples = _p(keep[-1])
        s.n_samples = keep[-1].shape[1]
    s.sample_t0, s.sample_dt = sysd.sample_t0, sysd.sample_dt
    return s


def _grid(g):
    o = or_grid()
    o.ta, o.dt, o.n_steps, o.n_sub = g.ta, g.dt, g.n_steps, g.n_sub
    return o


def free_propagators(system, grid):
    keep = []
    s = _system(system, keep)
    g = _grid(grid)
    N2 = system.dim ** 2
    M = np.zeros((max(1, 2 * grid.n_steps), N2, N2), dtype=np.complex128)
    lib().or_free_propagators(C.byref(s), C.byref(g), _p(M))
    return M[: 2 * grid.n_steps]


def expm(A):
    A = _c(A)
    E = np.zeros_like(A)
    lib().or_expm(C.c_int(A.shape[0]), _p(A), _p(E))
    return E


def propagate(system, grid, rho0, out_ops, traj, pt=None, M=None, nthreads=1, blocked=0):
    """Same contract as pyaceqd_amd.engine.propagate (list of (window, n_out) arrays); a list of systems
    with traj.system is handled by running each system's trajectories separately. blocked = bt > 0 runs
    or_propagate_blocked (pqd_oracle_blk.c: lockstep blocks of bt trajectories, bench.py's CPU baseline)."""
    from pyaceqd_amd.engine import split_output, Trajectories
    if isinstance(system, (list, tuple)):
        res = [None] * traj.n_traj
        sysidx = np.asarray(traj.system if traj.system is not None else np.zeros(traj.n_traj, dtype=int))
        for k, sy in enumerate(system):
            ids = np.nonzero(sysidx == k)[0]
            if len(ids) == 0:
                continue
            remap = {int(t): i for i, t in enumerate(ids)}
            sub = Trajectories(np.asarray(traj.out_begin)[ids], np.asarray(traj.out_end)[ids],
                               [type(m)(remap[m.traj], m.step, m.before, m.kind, m.op) for m in traj.mtos
                                if m.traj in remap])
            for i, r in zip(ids, propagate(sy, grid, rho0, out_ops, sub, pt=pt, nthreads=nthreads, blocked=blocked)):
                res[i] = r
        return res
    keep = []
    N = system.dim
    s = _system(system, keep)
    g = _grid(grid)
    ptc = None
    if pt is not None:
        ptc = or_pt()
        sched = pt.schedule(max(1, grid.n_steps))
        keep += [pt.Q, pt.closure, pt.closure0, pt.bond0, pt.gmap, sched]
        ptc.chi, ptc.D, ptc.n_slices = pt.chi, pt.D, pt.n_slices
        ptc.Q, ptc.closure, ptc.closure0, ptc.bond0 = _p(pt.Q), _p(pt.closure), _p(pt.closure0), _p(pt.bond0)
        ptc.gmap, ptc.sched = pt.gmap.ctypes.data_as(P_I32), sched.ctypes.data_as(P_I32)
    n_out = len(out_ops)
    ops = _c(np.stack([np.asarray(o).reshape(N, N) for o in out_ops]))
    r0 = _c(rho0).reshape(N * N)
    off, total = traj.offsets(n_out)
    t = or_traj()
    b = np.ascontiguousarray(traj.out_begin, dtype=np.int32)
    e = np.ascontiguousarray(traj.out_end, dtype=np.int32)
    keep += [b, e, off]
    t.n_traj, t.out_begin, t.out_end, t.out_offset = traj.n_traj, b.ctypes.data_as(P_I32), e.ctypes.data_as(P_I32), \
        off.ctypes.data_as(P_I64)
    t.n_mto = len(traj.mtos)
    if traj.mtos:
        arrs = [np.ascontiguousarray([getattr(m, f) if f != "before" else int(m.before) for m in traj.mtos],
                                     dtype=np.int32) for f in ("traj", "step", "before", "kind")]
        mo = _c(np.stack([np.asarray(m.op).reshape(N, N) for m in traj.mtos]))
        keep += arrs + [mo]
        t.mto_traj, t.mto_step, t.mto_before, t.mto_kind = [a.ctypes.data_as(P_I32) for a in arrs]
        t.mto_ops = _p(mo)
    out = np.zeros(max(1, total), dtype=np.complex128)
    Mp = None
    if M is not None:
        M = _c(M)
        keep.append(M)
        Mp = _p(M)
    args = (C.byref(s), C.byref(g), C.byref(ptc) if ptc is not None else None, _p(r0), C.c_int(n_out), _p(ops),
            C.byref(t), Mp, _p(out), C.c_int(nthreads))
    rc = lib().or_propagate_blocked(*args, C.c_int(blocked)) if blocked > 0 else lib().or_propagate(*args)
    assert rc == 0
    return split_output(out, traj, n_out)


# ---------------------------------------------------------------- map-chain restatements (Fortran layouts)
def _f(a):
    return np.asfortranarray(a, dtype=np.complex128)


def _r(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _fp(a):
    return a.ctypes.data_as(P_C)


def propagate_tau(dm_tl, rho_init, n_tau, dim, j_start):
    dm_tl, rho_init = _f(dm_tl), _f(rho_init)
    out = np.zeros((dim * dim, n_tau + 1), dtype=np.complex128, order="F")
    lib().or_propagate_tau(_fp(dm_tl), _fp(rho_init), C.c_int(n_tau), C.c_int(dim), C.c_int(j_start), _fp(out))
    return out


def calc_onetime_parallel(dm_tl, rho_init, n_tau, dim, opa, opb, opc, time, time_sparse, nthreads=1):
    dm_tl, rho_init = _f(dm_tl), _f(rho_init)
    opa, opb, opc = _f(opa), _f(opb), _f(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    out = np.zeros((len(time_sparse), n_tau + 1), dtype=np.complex128, order="F")
    lib().or_calc_onetime_parallel(_fp(dm_tl), _fp(rho_init), C.c_int(n_tau), C.c_int(len(time_sparse)),
                                   C.c_int(len(time)), C.c_int(dim), _fp(opa), _fp(opb), _fp(opc),
                                   time.ctypes.data_as(P_F), time_sparse.ctypes.data_as(P_F), _fp(out),
                                   C.c_int(nthreads))
    return out


def calc_onetime_parallel_block(dm_block, dm_s, rho_init, n_tb, nx_tau, dim, opa, opb, opc, time, time_sparse):
    dm_block, dm_s, rho_init = _f(dm_block), _f(dm_s), _f(rho_init)
    opa, opb, opc = _f(opa), _f(opb), _f(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    out = np.zeros((len(time_sparse), n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    lib().or_calc_onetime_parallel_block(_fp(dm_block), _fp(dm_s), _fp(rho_init), C.c_int(n_tb), C.c_int(nx_tau),
                                         C.c_int(dm_block.shape[2]), C.c_int(len(time_sparse)), C.c_int(len(time)),
                                         C.c_int(dim), _fp(opa), _fp(opb), _fp(opc), time.ctypes.data_as(P_F),
                                         time_sparse.ctypes.data_as(P_F), _fp(out))
    return out


def calc_twotime_phonon_block(dm_taucs2, dm_sep1, dm_sep2, dm_s, rho_init, n_tb, nx_tau, dim, opa, opb, opc, time,
                              time_sparse):
    dm_taucs2, dm_sep1, dm_sep2, dm_s = _f(dm_taucs2), _f(dm_sep1), _f(dm_sep2), _f(dm_s)
    rho_init = _f(rho_init)
    opa, opb, opc = _f(opa), _f(opb), _f(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    out = np.zeros((len(time_sparse), n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    lib().or_calc_twotime_phonon_block(_fp(dm_taucs2), _fp(dm_sep1), _fp(dm_sep2), _fp(dm_s), _fp(rho_init),
                                       C.c_int(n_tb), C.c_int(nx_tau), C.c_int(dm_sep1.shape[2]),
                                       C.c_int(len(time_sparse)), C.c_int(len(time)), C.c_int(dm_taucs2.shape[2]),
                                       C.c_int(dim), _fp(opa), _fp(opb), _fp(opc), time.ctypes.data_as(P_F),
                                       time_sparse.ctypes.data_as(P_F), _fp(out))
    return out


def four_time_8op(dm_1, dm_2, rho_init, t1, precalc, dt, dim, ops8, early_only, late_t1_only, tb):
    dm_1, dm_2, precalc, rho_init = _f(dm_1), _f(dm_2), _f(precalc), _f(rho_init)
    ops = np.ascontiguousarray(np.stack([_f(o).reshape(dim * dim, order="F") for o in ops8]))
    t1 = _r(t1)
    out = np.zeros((len(t1), len(t1)), dtype=np.complex128, order="F")
    lib().or_four_time_8op(_fp(dm_1), _fp(dm_2), _fp(rho_init), t1.ctypes.data_as(P_F), _fp(precalc),
                           C.c_int(len(t1)), C.c_double(dt), C.c_int(dm_1.shape[2]), C.c_int(dim), _fp(ops),
                           C.c_int(int(early_only)), C.c_int(int(late_t1_only)), C.c_double(tb),
                           C.c_int(precalc.shape[2]), _fp(out))
    return out


def four_time(dm_1, dm_2, rho_init, t1, precalc, dt, dim, ops4, tb):
    dm_1, dm_2, precalc, rho_init = _f(dm_1), _f(dm_2), _f(precalc), _f(rho_init)
    ops = np.ascontiguousarray(np.stack([_f(o).reshape(dim * dim, order="F") for o in ops4]))
    t1 = _r(t1)
    out = np.zeros((len(t1), len(t1)), dtype=np.complex128, order="F")
    lib().or_four_time(_fp(dm_1), _fp(dm_2), _fp(rho_init), t1.ctypes.data_as(P_F), _fp(precalc), C.c_int(len(t1)),
                       C.c_double(dt), C.c_int(dm_1.shape[2]), C.c_int(dim), _fp(ops), C.c_double(tb),
                       C.c_int(precalc.shape[2]), _fp(out))
    return out


def dynamics_t1(dm_1, dm_2, rho_init, t1, precalc, dt, dim, tb):
    dm_1, dm_2, precalc, rho_init = _f(dm_1), _f(dm_2), _f(precalc), _f(rho_init)
    t1 = _r(t1)
    out = np.zeros((dim * dim, 2 * len(t1) - 1), dtype=np.complex128, order="F")
    lib().or_dynamics_t1(_fp(dm_1), _fp(dm_2), _fp(rho_init), t1.ctypes.data_as(P_F), _fp(precalc), C.c_int(len(t1)),
                         C.c_double(dt), C.c_int(dm_1.shape[2]), C.c_int(dim), C.c_double(tb),
                         C.c_int(precalc.shape[2]), _fp(out))
    return out


def map_tail(M, X, w, n_steps):
    """checker for pqd_map_tail: the reference's own loop (two_time/correlations.py:866-1011, `for j: X = tl_map2 @ X;
    G[:, n_tauc + j + 1] = Bt @ X`), X with one column per row. Returns (n_x, n_steps)."""
    X = np.array(X, dtype=np.complex128, copy=True)
    out = np.zeros((X.shape[1], max(0, int(n_steps))), dtype=np.complex128)
    for j in range(int(n_steps)):
        X = M @ X
        out[:, j] = w @ X
    return out


def tl_dynmap_pseudo(dm, n_out=None, rcond=1e-12):
    """time-local maps out[i] = dm[i] pinv(dm[i-1], rcond), out[0] = dm[0] — numpy restatement of
    calc_tl_dynmap_pseudo (reference pyaceqd/tools.py:446-484, LAPACK SVD inside numpy's pinv)"""
    n_out = len(dm) if n_out is None else n_out
    out = np.empty((n_out,) + dm.shape[1:], dtype=np.complex128)
    out[0] = dm[0]
    for i in range(1, n_out):
        out[i] = dm[i] @ np.linalg.pinv(dm[i - 1], rcond=rcond)
    return out
