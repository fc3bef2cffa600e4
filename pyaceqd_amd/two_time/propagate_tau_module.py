"""Drop-in for the reference's f2py module `propagate_tau_module` (two_time/propagate_tau.f90), on libpqd.

Same function names, positional order and keywords as the f2py wrappers the reference calls
(correlations.py:534/583/782/831, purity.py:602/709/741/770): Fortran-ordered complex128 inputs,
hidden dimensions optional (inferred from the shapes, as f2py does), results returned Fortran-ordered.
"""
import numpy as np

from .. import _lib

_c = lambda a: np.asfortranarray(a, dtype=np.complex128)  # noqa: E731
_r = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731


def _p(a):
    # Fortran-ordered complex array -> pointer to its column-major buffer
    return a.ctypes.data_as(_lib.P_C128)


def _ctx():
    return _lib.context()


def propagate_tau(dm_tl, rho_init, n_tau, dim, j_start):
    """rho_out(:, k+1) = dm_tl(:, :, j_start + k) rho_out(:, k)   (propagate_tau.f90:3-19)"""
    dm_tl, rho_init = _c(dm_tl), _c(rho_init)
    N2 = dim * dim
    n_maps = dm_tl.shape[2] if dm_tl.ndim == 3 else 1
    out = np.zeros((N2, n_tau + 1), dtype=np.complex128, order="F")
    ctx = _ctx()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_propagate_tau(ctx.handle, _p(dm_tl), int(n_maps), _p(rho_init), int(n_tau),
                                                int(dim), int(j_start), _p(out)))
    return out


def map_tail(M, X, w, n_steps):
    """G[i, j] = w . M^{j+1} x_i (i < n_x = X.shape[1], j < n_steps) on the GPU (pqd_map_tail): the tau tails of the
    phonon dynamical-map correlations (correlations.py:866-1186: `X = tl_map2 @ X; G[:, n_tauc + j + 1] = Bt @ X`),
    X with one column per row i (the reference's layout). Returns (n_x, n_steps) complex."""
    M = np.ascontiguousarray(M, dtype=np.complex128)
    Xr = np.ascontiguousarray(np.asarray(X, dtype=np.complex128).T)        # [n_x][N2]
    w = np.ascontiguousarray(w, dtype=np.complex128)
    n_x, N2 = Xr.shape
    out = np.zeros((n_x, max(0, int(n_steps))), dtype=np.complex128)
    if n_x == 0 or n_steps <= 0:
        return out
    ctx = _ctx()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_map_tail(ctx.handle, _lib.cptr(M), int(N2), _lib.cptr(Xr), int(n_x), _lib.cptr(w),
                                           int(n_steps), _lib.cptr(out)))
    return out


def calc_onetime_parallel(dm_tl, rho_init, n_tau, dim, opa, opb, opc, time, time_sparse, n_t=None, n_tfull=None):
    """G(t_i, tau_k) on the dynamical-map chain (propagate_tau.f90:110-187)"""
    dm_tl, rho_init = _c(dm_tl), _c(rho_init)
    opa, opb, opc = _c(opa), _c(opb), _c(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    n_t = len(time_sparse) if n_t is None else n_t
    n_tfull = len(time) if n_tfull is None else n_tfull
    if dm_tl.shape[2] < n_tfull - 1:
        raise ValueError(f"dm_tl has {dm_tl.shape[2]} maps, need n_tfull-1 = {n_tfull - 1}")
    out = np.zeros((n_t, n_tau + 1), dtype=np.complex128, order="F")
    ctx = _ctx()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_calc_onetime_parallel(
            ctx.handle, _p(dm_tl), _p(rho_init), int(n_tau), int(n_t), int(n_tfull), int(dim), _p(opa), _p(opb),
            _p(opc), _lib.fptr(time), _lib.fptr(time_sparse), _p(out)))
    return out


def calc_onetime_parallel_block(dm_block, dm_s, rho_init, n_tb, nx_tau, dim, opa, opb, opc, time, time_sparse,
                                n_map=None, n_t=None, n_tfull=None):
    """periodic map blocks + stationary map (propagate_tau.f90:189-295)"""
    dm_block, dm_s, rho_init = _c(dm_block), _c(dm_s), _c(rho_init)
    opa, opb, opc = _c(opa), _c(opb), _c(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    n_map = dm_block.shape[2] if n_map is None else n_map
    n_t = len(time_sparse) if n_t is None else n_t
    n_tfull = len(time) if n_tfull is None else n_tfull
    out = np.zeros((n_t, n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    ctx = _ctx()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_calc_onetime_parallel_block(
            ctx.handle, _p(dm_block), _p(dm_s), _p(rho_init), int(n_tb), int(nx_tau), int(n_map), int(n_t),
            int(n_tfull), int(dim), _p(opa), _p(opb), _p(opc), _lib.fptr(time), _lib.fptr(time_sparse), _p(out)))
    return out


def calc_twotime_phonon_block(dm_taucs2, dm_sep1, dm_sep2, dm_s, rho_init, n_tb, nx_tau, dim, opa, opb, opc, time,
                              time_sparse, n_map=None, n_t=None, n_tfull=None, n_tauc=None):
    """two-time phonon-block sweep with transpose(opB) traces (propagate_tau.f90:374-536)"""
    dm_taucs2, dm_sep1, dm_sep2, dm_s = _c(dm_taucs2), _c(dm_sep1), _c(dm_sep2), _c(dm_s)
    rho_init = _c(rho_init)
    opa, opb, opc = _c(opa), _c(opb), _c(opc)
    time, time_sparse = _r(time), _r(time_sparse)
    n_map = dm_sep1.shape[2] if n_map is None else n_map
    n_tauc = dm_taucs2.shape[2] if n_tauc is None else n_tauc
    n_t = len(time_sparse) if n_t is None else n_t
    n_tfull = len(time) if n_tfull is None else n_tfull
    out = np.zeros((n_t, n_tb * nx_tau + 1), dtype=np.complex128, order="F")
    ctx = _ctx()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_calc_twotime_phonon_block(
            ctx.handle, _p(dm_taucs2), _p(dm_sep1), _p(dm_sep2), _p(dm_s), _p(rho_init), int(n_tb), int(nx_tau),
            int(n_map), int(n_t), int(n_tfull), int(n_tauc), int(dim), _p(opa), _p(opb), _p(opc),
            _lib.fptr(time), _lib.fptr(time_sparse), _p(out)))
    return out
