"""Drop-in for the reference's f2py module `timebin_tl` (timebin/timebin_tl.f90), on libpqd.

Same names and argument order as the calls in timebin/twophoton_new.py:661/697/712: map stacks
Fortran-ordered (N^2, N^2, n) exactly as the caller builds them (including its conj-transposed feed,
twophoton_new.py:114-116); hidden dimensions optional.
"""
import numpy as np

from .. import _lib

_c = lambda a: np.asfortranarray(a, dtype=np.complex128)  # noqa: E731
_r = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731


def _p(a):
    return a.ctypes.data_as(_lib.P_C128)


def four_time_8op(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, op_et1l, op_et1r, op_et2l, op_et2r,
                  op_lt1l, op_lt1r, op_lt2l, op_lt2r, early_only, late_t1_only, tb,
                  n_t=None, n_map=None, n_precalc=None, rows=None):
    """four-time correlation over the (t1, t2 >= t1) triangle (timebin_tl.f90:216-303). `rows=(lo, hi)` (an extension
    for sharding, four_time_8op_sharded) computes only the rows i in [lo, hi); the other elements stay 0."""
    dm_1, dm_2, precalc_tls, rho_init = _c(dm_1), _c(dm_2), _c(precalc_tls), _c(rho_init)
    t1 = _r(t1)
    ops = np.ascontiguousarray(np.stack([_c(o).reshape(dim * dim, order="F") for o in
                                         (op_et1l, op_et1r, op_et2l, op_et2r, op_lt1l, op_lt1r, op_lt2l, op_lt2r)]))
    n_t = len(t1) if n_t is None else n_t
    n_map = dm_1.shape[2] if n_map is None else n_map
    n_precalc = precalc_tls.shape[2] if n_precalc is None else n_precalc
    out = np.zeros((n_t, n_t), dtype=np.complex128, order="F")
    ctx = _lib.context()
    args = (ctx.handle, _p(dm_1), _p(dm_2), _p(rho_init), _lib.fptr(t1), _p(precalc_tls), int(n_t), float(dt),
            int(n_map), int(dim), ops.ctypes.data_as(_lib.P_C128), int(bool(early_only)), int(bool(late_t1_only)),
            float(tb), int(n_precalc))
    with ctx.lock:
        if rows is None:
            _lib.check(_lib.lib().pqd_four_time_8op(*args, _p(out)))
        else:
            _lib.check(_lib.lib().pqd_four_time_8op_rows(*args, int(rows[0]), int(rows[1]), _p(out)))
    return out


def four_time_8op_sharded(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, op_et1l, op_et1r, op_et2l, op_et2r,
                          op_lt1l, op_lt1r, op_lt2l, op_lt2r, early_only, late_t1_only, tb, dist=None, dst=0):
    """four_time_8op over the ranks of `dist` (one process per GPU): rank r computes the rows
    scan.triangular_rows(n_t, r, world) of the pair triangle (about the same number of (i, j) pairs per rank; the
    reference's OpenMP loop over i, timebin_tl.f90:255-302, split across GPUs), packs each of its rows' pairs
    G(i, i..n_t-1) into one tensor and scan.gather_tensor sends the blocks to `dst` (RCCL point-to-point; gloo with host
    tensors), which unpacks them into the (n_t, n_t) result. Returns the same array as four_time_8op on `dst` (bit for
    bit: every element is computed by exactly one rank with the same kernel), None on the other ranks."""
    from ..scan import gather_tensor, triangular_rows
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return four_time_8op(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, op_et1l, op_et1r, op_et2l, op_et2r,
                             op_lt1l, op_lt1r, op_lt2l, op_lt2r, early_only, late_t1_only, tb)
    import torch
    n_t = len(t1)
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = triangular_rows(n_t, rank, world)
    part = four_time_8op(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, op_et1l, op_et1r, op_et2l, op_et2r,
                         op_lt1l, op_lt1r, op_lt2l, op_lt2r, early_only, late_t1_only, tb, rows=(lo, hi))
    packed = np.concatenate([part[i, i:] for i in range(lo, hi)]) if hi > lo else np.zeros(0, np.complex128)
    on_dev = dist.get_backend() != "gloo" and torch.cuda.is_available()
    dev = f"cuda:{torch.cuda.current_device()}" if on_dev else "cpu"
    allp = gather_tensor(torch.from_numpy(np.ascontiguousarray(packed)).to(dev), dist, dst=dst)
    if rank != dst:
        return None
    allp = allp.cpu().numpy()
    out = np.zeros((n_t, n_t), dtype=np.complex128, order="F")
    o = 0
    for i in range(n_t):
        out[i, i:] = allp[o: o + n_t - i]
        o += n_t - i
    if o != allp.size:
        raise RuntimeError(f"gathered {allp.size} pairs, expected {o}")
    return out


def four_time(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, op_1, op_2, op_3, op_4, tb,
              n_t=None, n_map=None, n_precalc=None):
    """four-operator variant (timebin_tl.f90:145-214)"""
    dm_1, dm_2, precalc_tls, rho_init = _c(dm_1), _c(dm_2), _c(precalc_tls), _c(rho_init)
    t1 = _r(t1)
    ops = np.ascontiguousarray(np.stack([_c(o).reshape(dim * dim, order="F") for o in (op_1, op_2, op_3, op_4)]))
    n_t = len(t1) if n_t is None else n_t
    n_map = dm_1.shape[2] if n_map is None else n_map
    n_precalc = precalc_tls.shape[2] if n_precalc is None else n_precalc
    out = np.zeros((n_t, n_t), dtype=np.complex128, order="F")
    ctx = _lib.context()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_four_time(
            ctx.handle, _p(dm_1), _p(dm_2), _p(rho_init), _lib.fptr(t1), _p(precalc_tls), int(n_t), float(dt),
            int(n_map), int(dim), ops.ctypes.data_as(_lib.P_C128), float(tb), int(n_precalc), _p(out)))
    return out


def dynamics_t1(dm_1, dm_2, rho_init, t1, precalc_tls, dt, dim, tb, n_t=None, n_map=None, n_precalc=None):
    """rho along the t1 grid, first with dm_1 then with dm_2 (timebin_tl.f90:305-342)"""
    dm_1, dm_2, precalc_tls, rho_init = _c(dm_1), _c(dm_2), _c(precalc_tls), _c(rho_init)
    t1 = _r(t1)
    n_t = len(t1) if n_t is None else n_t
    n_map = dm_1.shape[2] if n_map is None else n_map
    n_precalc = precalc_tls.shape[2] if n_precalc is None else n_precalc
    out = np.zeros((dim * dim, 2 * n_t - 1), dtype=np.complex128, order="F")
    ctx = _lib.context()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_dynamics_t1(
            ctx.handle, _p(dm_1), _p(dm_2), _p(rho_init), _lib.fptr(t1), _p(precalc_tls), int(n_t), float(dt),
            int(n_map), int(dim), float(tb), int(n_precalc), _p(out)))
    return out


class utils:
    """timebin_tl.utils: propagate_tb / fast_propagate (timebin_tl.f90:23-77) through dynamics_t1."""

    @staticmethod
    def propagate_tb(t_start, t_stop, dt, rho, dm_tl, dm_tl_precalc, n_precalc=None, dimsquare=None, n_dm=None):
        dim = int(round(np.sqrt(len(rho))))
        r = dynamics_t1(dm_tl, dm_tl, rho, np.array([t_start, t_stop]), dm_tl_precalc, dt, dim, 0.0)
        return np.asarray(r[:, 1])

    @staticmethod
    def fast_propagate(rho, dm_tl_precalc, n_steps, dimsquare=None, n_precalc=None):
        dm = np.asfortranarray(dm_tl_precalc, dtype=np.complex128)
        dim = int(round(np.sqrt(len(rho))))
        dt = 1.0
        # start past the explicit maps so only the binary powers are used
        n_dm = dm.shape[2]
        r = dynamics_t1(dm, dm, rho, np.array([float(n_dm), float(n_dm + n_steps)]), dm, dt, dim, 0.0)
        return np.asarray(r[:, 1])
