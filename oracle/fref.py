"""ctypes bindings to the reference's OWN Fortran sweep kernels, built from
/root/reference/pyaceqd/two_time/propagate_tau.f90 and .../timebin/timebin_tl.f90 by
oracle/Makefile into oracle/_ref/.  TEST INFRASTRUCTURE ONLY: used to generate and
re-check golden vectors and as the "reference" CPU baseline for the map-chain sweeps.

Every function passes the Fortran arguments in their declared order (all by reference),
with the f2py-hidden dimensions made explicit, exactly as the reference signatures read:
  propagate_tau          propagate_tau.f90:3
  calc_onetime_parallel  propagate_tau.f90:110
  calc_onetime_parallel_block  propagate_tau.f90:189
  calc_twotime_phonon_block    propagate_tau.f90:374
  four_time              timebin_tl.f90:145
  four_time_8op          timebin_tl.f90:216
  dynamics_t1            timebin_tl.f90:305
  dynamics_t1_t2         timebin_tl.f90:344
"""
import ctypes as C
import os
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REF = os.path.join(_HERE, "_ref")


def available():
    return (os.path.exists(os.path.join(_REF, "libfref_tau.so"))
            and os.path.exists(os.path.join(_REF, "libfref_tb.so")))


_tau = None
_tb = None


def _libs():
    global _tau, _tb
    if _tau is None:
        _tau = C.CDLL(os.path.join(_REF, "libfref_tau.so"))
        _tb = C.CDLL(os.path.join(_REF, "libfref_tb.so"))
    return _tau, _tb


def _i(v):
    return C.byref(C.c_int(int(v)))


def _d(v):
    return C.byref(C.c_double(float(v)))


def _l(v):
    # flang LOGICAL(4): .true. = 1
    return C.byref(C.c_int(1 if v else 0))


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _cf(a):
    return np.asfortranarray(a, dtype=np.complex128)


def _rf(a):
    return np.asfortranarray(a, dtype=np.float64)


def propagate_tau(dm_tl, rho_init, n_tau, dim, j_start):
    lib, _ = _libs()
    dm_tl = _cf(dm_tl); rho_init = _cf(rho_init)
    out = np.zeros((dim * dim, n_tau + 1), dtype=np.complex128, order="F")
    lib.propagate_tau_(_p(dm_tl), _p(rho_init), _i(n_tau), _i(dim), _i(j_start), _p(out))
    return out


def calc_onetime_parallel(dm_tl, rho_init, n_tau, dim, opa, opb, opc, time, time_sparse):
    lib, _ = _libs()
    dm_tl = _cf(dm_tl); rho_init = _cf(rho_init)
    opa, opb, opc = _cf(opa), _cf(opb), _cf(opc)
    time = _rf(time); time_sparse = _rf(time_sparse)
    n_t, n_tfull = len(time_sparse), len(time)
    out = np.zeros((n_t, n_tau + 1), dtype=np.complex128, order="F")
    lib.calc_onetime_parallel_(_p(dm_tl), _p(rho_init), _i(n_tau), _i(n_t), _i(n_tfull), _i(dim),
                               _p(opa), _p(opb), _p(opc), _p(time), _p(time_sparse), _p(out))
    return out


def calc_onetime_parallel_block(dm_block, dm_s, rho_init, n_tb, nx_tau, dim, opa, opb, opc, time, time_sparse):
    lib, _ = _libs()
    dm_block = _cf(dm_block); dm_s = _cf(dm_s); rho_init = _cf(rho_init)
    opa, opb, opc = _cf(opa), _cf(opb), _cf(opc)
    time = _rf(time); time_sparse = _rf(time_sparse)
    n_map = dm_block.shape[2]
    n_t, n_tfull = len(time_sparse), len(time)
    out = np.zeros((n_t, n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    lib.calc_onetime_parallel_block_(_p(dm_block), _p(dm_s), _p(rho_init), _i(n_tb), _i(nx_tau), _i(n_map),
                                     _i(n_t), _i(n_tfull), _i(dim), _p(opa), _p(opb), _p(opc),
                                     _p(time), _p(time_sparse), _p(out))
    return out


def calc_twotime_phonon_block(dm_taucs2, dm_sep1, dm_sep2, dm_s, rho_init, n_tb, nx_tau, dim,
                              opa, opb, opc, time, time_sparse):
    lib, _ = _libs()
    dm_taucs2 = _cf(dm_taucs2); dm_sep1 = _cf(dm_sep1); dm_sep2 = _cf(dm_sep2); dm_s = _cf(dm_s)
    rho_init = _cf(rho_init)
    opa, opb, opc = _cf(opa), _cf(opb), _cf(opc)
    time = _rf(time); time_sparse = _rf(time_sparse)
    n_map = dm_sep1.shape[2]
    n_tauc = dm_taucs2.shape[2]
    n_t, n_tfull = len(time_sparse), len(time)
    out = np.zeros((n_t, n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    lib.calc_twotime_phonon_block_(_p(dm_taucs2), _p(dm_sep1), _p(dm_sep2), _p(dm_s), _p(rho_init),
                                   _i(n_tb), _i(nx_tau), _i(n_map), _i(n_t), _i(n_tfull), _i(n_tauc), _i(dim),
                                   _p(opa), _p(opb), _p(opc), _p(time), _p(time_sparse), _p(out))
    return out


def four_time(dm_1, dm_2, rho_init, t1, precalc, dt, dim, op1, op2, op3, op4, tb):
    _, lib = _libs()
    dm_1, dm_2, precalc, rho_init = _cf(dm_1), _cf(dm_2), _cf(precalc), _cf(rho_init)
    ops = [_cf(o) for o in (op1, op2, op3, op4)]
    t1 = _rf(t1)
    n_t, n_map, n_precalc = len(t1), dm_1.shape[2], precalc.shape[2]
    out = np.zeros((n_t, n_t), dtype=np.complex128, order="F")
    lib.four_time_(_p(dm_1), _p(dm_2), _p(rho_init), _p(t1), _p(precalc), _i(n_t), _d(dt), _i(n_map), _i(dim),
                   *[_p(o) for o in ops], _d(tb), _i(n_precalc), _p(out))
    return out


def four_time_8op(dm_1, dm_2, rho_init, t1, precalc, dt, dim, ops8, early_only, late_t1_only, tb):
    _, lib = _libs()
    dm_1, dm_2, precalc, rho_init = _cf(dm_1), _cf(dm_2), _cf(precalc), _cf(rho_init)
    ops = [_cf(o) for o in ops8]
    t1 = _rf(t1)
    n_t, n_map, n_precalc = len(t1), dm_1.shape[2], precalc.shape[2]
    out = np.zeros((n_t, n_t), dtype=np.complex128, order="F")
    lib.four_time_8op_(_p(dm_1), _p(dm_2), _p(rho_init), _p(t1), _p(precalc), _i(n_t), _d(dt), _i(n_map), _i(dim),
                       *[_p(o) for o in ops], _l(early_only), _l(late_t1_only), _d(tb), _i(n_precalc), _p(out))
    return out


def dynamics_t1(dm_1, dm_2, rho_init, t1, precalc, dt, dim, tb):
    _, lib = _libs()
    dm_1, dm_2, precalc, rho_init = _cf(dm_1), _cf(dm_2), _cf(precalc), _cf(rho_init)
    t1 = _rf(t1)
    n_t, n_map, n_precalc = len(t1), dm_1.shape[2], precalc.shape[2]
    out = np.zeros((dim * dim, 2 * n_t - 1), dtype=np.complex128, order="F")
    lib.dynamics_t1_(_p(dm_1), _p(dm_2), _p(rho_init), _p(t1), _p(precalc), _i(n_t), _d(dt), _i(n_map), _i(dim),
                     _d(tb), _i(n_precalc), _p(out))
    return out
