"""Helpers either side of the propagator: time grids, density-matrix assembly, dynamical-map utilities.

Same names and semantics as the hot-path parts of pyaceqd/tools.py (time grids :9-135, export_csv
:137, concurrence :167, compose_dm :188, output_ops_dm :248, op_to_matrix :260,
calc_tl_dynmap_pseudo :446, extract_dms :486, use_tl_map :567, use_dm_block :590,
tl_pad_stationary(_nsteps) :610/:620, use_tl_map_mto :630). Pinned against the reference's own
outputs in tests/golden/pyref_tools.npz. Plotting/calibration helpers of the reference are out of
scope.
"""
import itertools

import numpy as np

from . import opgrammar


# ----------------------------------------------------------------------------------------- time grids
def _merge_intervals(intervals):
    """Merge sorted [start, end] intervals that overlap or touch (in place, returns the list)."""
    k = 0
    while k < len(intervals) - 1:
        if intervals[k][1] >= intervals[k + 1][0]:
            intervals[k][1] = max(intervals[k][1], intervals[k + 1][1])
            del intervals[k + 1]
            k = 0
            continue
        k += 1
    return intervals


def get_gaussian_t(t0, tend, *pulses, dt_max=1.0, dt_min=0.01, interval_per_step=0.05):
    """Adaptive grid: a new point whenever the accumulated pulse area reaches interval_per_step
    (or dt_max has passed), probing on a dt_min raster."""
    probe = np.arange(t0, tend, dt_min)
    area = lambda t: np.sum([p.get_integral(t) for p in pulses])  # noqa: E731
    pts = [t0]
    n_cap = int(dt_max / dt_min)
    since, acc = 0, 0.0
    prev = area(probe[0]) if len(probe) else 0.0
    for t in probe[1:]:
        cur = area(t)
        acc += cur - prev
        prev = cur
        since += 1
        if acc >= interval_per_step or since == n_cap:
            pts.append(t)
            since, acc = 0, 0.0
    return np.array(pts)


def construct_t(t0, tend, dt_small=0.1, dt_big=1.0, dt_exp=None, *pulses, factor_tau=4, simple_exp=False,
                gaussian_t=False, add_tend=True):
    """Fine steps (dt_small) within factor_tau*tau of every pulse centre, dt_big elsewhere."""
    if dt_exp is None:
        dt_exp = dt_small
    windows = []
    for p in pulses:
        if t0 < p.t0 < tend:
            windows.append([p.t0 - factor_tau * p.tau, p.t0 + factor_tau * p.tau])
        else:
            if p.t0 > tend:
                print("WARNING: tend is smaller than the end of a pulse")
            if p.t0 < t0:
                print("WARNING: t0 is greater than the start of a pulse")
    windows = _merge_intervals(sorted(windows))
    if windows[0][0] < t0:
        print("WARNING: t0 is greater than the start of the first pulse")
    if windows[-1][1] > tend:
        print("WARNING: tend is smaller than the end of the last pulse")
    parts = [np.arange(t0, windows[0][0], dt_big)]
    if simple_exp and len(windows) == 1 and windows[0][1] != 0:
        a, b = windows[0]
        if gaussian_t:
            parts.append(get_gaussian_t(a, b, *pulses, dt_max=dt_big, dt_min=dt_small, interval_per_step=0.05))
        else:
            parts.append(np.arange(a, b, dt_small))
        parts.append(np.round(np.exp(np.arange(np.log(b), np.log(tend), dt_exp))))
        parts.append(np.array([tend]))
        return np.concatenate(parts)
    for k, (a, b) in enumerate(windows):
        if k:
            parts.append(np.arange(windows[k - 1][1], a, dt_big))
        parts.append(np.arange(a, b, dt_small))
    parts.append(np.arange(windows[-1][1], tend, dt_big))
    if add_tend:
        parts.append(np.array([tend]))
    return np.concatenate(parts)


def round_to_dt(t, dt):
    """Round to the dt raster, dropping duplicates (first occurrence order kept)."""
    r = np.round(t / dt) * dt
    _, first = np.unique(r, return_index=True)
    return r[np.sort(first)]


def simple_t_gaussian(t0, texp, tend, dt_small=0.1, dt_big=1.0, *pulses, decimals=2, exp_part=True, add_tend=True):
    """Adaptive grid over [t0, texp), then exponential (or dt_big) spacing up to tend, on the dt_small raster."""
    parts = [get_gaussian_t(t0, texp, *pulses, dt_max=dt_big, dt_min=dt_small, interval_per_step=0.05)]
    if exp_part:
        parts.append(np.exp(np.arange(np.log(texp - t0), np.log(tend - t0), dt_small)) + t0)
    else:
        parts.append(np.arange(texp, tend, dt_big))
    if add_tend:
        parts.append(np.array([tend]))
    return round_to_dt(np.concatenate(parts), dt_small)


def export_csv(filename, *arg, precision=4, delimit=",", verbose=False):
    """Columns -> text file with fixed decimals (the pulse-file format is precision=8, delimit=' ')."""
    np.savetxt(filename, np.c_[arg], fmt=["%.{}f".format(precision)] * len(arg), delimiter=delimit, newline="\n")
    if verbose:
        print("[i] csv saved to {}".format(filename))


# ----------------------------------------------------------------------------- density matrices
def concurrence(rho):
    """Wootters concurrence of a two-qubit density matrix (tools.py:167-172). A non-physical input with a negative
    eigenvalue of rho T rho* T gives NaN, as in the reference (np.max propagates it; builtin max would not)."""
    flip = np.fliplr(np.diag([-1.0, 1.0, 1.0, -1.0]))
    R = rho @ flip @ np.conjugate(rho) @ flip
    with np.errstate(invalid="ignore"):
        lam = np.sqrt(np.sort(np.real(np.linalg.eigvals(R))))
    return np.max([0.0, lam[-1] - np.sum(lam[:-1])])


def compose_dm(outputs, dim=2):
    """Upper-triangle outputs (time axis first) -> (t, rho[n_t, dim, dim])."""
    n_t = len(outputs[0])
    rho = np.zeros((n_t, dim, dim), dtype=np.complex128)
    iu = [(j, k) for j in range(dim) for k in range(j, dim)]
    for n, (j, k) in enumerate(iu, start=1):
        rho[:, j, k] = outputs[n]
        rho[:, k, j] = np.conjugate(outputs[n])
    return np.real(outputs[0]), rho


def generate_basis_states(dim):
    return list(itertools.product(*[range(d) for d in dim]))


def basis_states(dim):
    dim = dim if isinstance(dim, list) else [dim]
    return ["|" + ",".join(str(i) for i in s) + "⟩" for s in generate_basis_states(dim)]


def matrix_element_operators(basis, dim, readable=False):
    ops = []
    for a in range(len(basis)):
        for b in range(a, len(basis)):
            if readable:
                parts = [f"|{x}⟩⟨{y}|_{dim[k]}" for k, (x, y) in enumerate(zip(basis[a], basis[b]))]
                ops.append(" ⊗ ".join(parts))
            else:
                parts = [f"|{x}><{y}|_{dim[k]}" for k, (x, y) in enumerate(zip(basis[a], basis[b]))]
                ops.append(" otimes ".join(parts))
    return ops


def output_ops_dm(dim=[2, 2], readable=False):
    """Output operators for every upper-triangle matrix element (compose_dm reassembles them)."""
    if not isinstance(dim, (list, tuple)):
        dim = [dim]
    dim = list(dim)
    return matrix_element_operators(generate_basis_states(dim), dim, readable=readable)


def op_to_matrix(op):
    """Operator string -> matrix (full ACE grammar via opgrammar, not only single |n><m|_d terms)."""
    return opgrammar.to_matrix(op)


# ------------------------------------------------------------------------- dynamical maps
def calc_tl_dynmap_pseudo(dm, times, debug=False):
    """Time-local maps E(t_{i+1}, t_i) = E(t_{i+1}, t0) pinv(E(t_i, t0)) from cumulative maps dm[i] = E(t_{i+1}, t0)
    (reference tools.py:446-484): out[0] = dm[0], out[i] = dm[i] pinv(dm[i-1], rcond=1e-12), len(times)-1 maps.

    Runs on the GPU (libpqd `pqd_tl_dynmap_pseudo`: one Jacobi SVD per map, one workgroup each). The reference's
    LinAlgError retry without rcond has no counterpart: the Jacobi SVD does not fail to converge; `debug` is
    accepted for signature compatibility."""
    from . import _lib
    dm = np.ascontiguousarray(dm, dtype=np.complex128)
    n_out = len(times) - 1
    if dm.ndim != 3 or dm.shape[1] != dm.shape[2]:
        raise ValueError(f"dm must be (n_t, n, n), got {dm.shape}")
    if n_out < 1 or dm.shape[0] < n_out:
        raise ValueError(f"need len(times)-1 = {n_out} >= 1 maps, dm has {dm.shape[0]}")
    dm = np.ascontiguousarray(dm[:n_out])
    out = np.empty_like(dm)
    ctx = _lib.context()
    with ctx.lock:
        _lib.check(_lib.lib().pqd_tl_dynmap_pseudo(ctx.handle, _lib.cptr(dm), int(n_out), int(dm.shape[1]),
                                                   1e-12, _lib.cptr(out)))
    return out


def extract_dms(dm, times, tau_c, t_MTOs):
    """Split maps into the first memory window, the windows starting at each MTO time, and the time-local map."""
    i_tl = int(np.where(times > times[0] + tau_c)[0][0])
    blocks = [dm[:i_tl]]
    for t in t_MTOs:
        hit = np.where(times == t)[0]
        if len(hit) == 0:
            print(f"Available times: {times}")
            print(f"Requested t_MTO: {t}")
            raise ValueError(f"t_MTO {t} not found in times array. Make sure that t_MTO is included in the times array.")
        blocks.append(dm[hit[0]: hit[0] + i_tl])
    return dm[i_tl], blocks


def check_tl_map_params(tl_map, rho0):
    n = int(rho0.shape[0])
    if rho0.shape[1] != n:
        raise ValueError("rho0 must be a {n}x{n} matrix")
    if tl_map.shape != (n ** 2, n ** 2):
        raise ValueError("tl_map must be a {}x{} matrix, is {}".format(n ** 2, n ** 2, np.shape(tl_map)))
    return n


def _chain(maps_for_step, n_steps, rho_first, n):
    rho = np.zeros((n_steps, n * n), dtype=complex)
    rho[0] = rho_first
    for i in range(n_steps - 1):
        rho[i + 1] = maps_for_step(i) @ rho[i]
    return rho


def use_tl_map(tl_map, times, rho0):
    n = check_tl_map_params(tl_map, rho0)
    return _chain(lambda i: tl_map, len(times), rho0.reshape(n * n), n).reshape(len(times), n, n)


def use_dm_block(dm, rho0):
    n = check_tl_map_params(dm[0], rho0)
    return _chain(lambda i: dm[i], len(dm) + 1, rho0.reshape(n * n), n).reshape(len(dm) + 1, n, n)


def tl_pad_stationary(tl_map, times, rho):
    n = check_tl_map_params(tl_map, rho[0])
    out = np.zeros((len(times), n * n), dtype=complex)
    out[: len(rho)] = rho.reshape(len(rho), n * n)
    for i in range(len(rho), len(times)):
        out[i] = tl_map @ out[i - 1]
    return out.reshape(len(times), n, n)


def tl_pad_stationary_nsteps(tl_map, n_steps, rho):
    n = check_tl_map_params(tl_map, rho)
    out = np.zeros((n_steps, n * n), dtype=complex)
    out[: len(rho)] = rho.reshape(-1, n * n)[: n_steps]
    for i in range(len(rho), n_steps):
        out[i] = tl_map @ out[i - 1]
    return out.reshape(n_steps, n, n)


def use_tl_map_mto(tl_map, dm_1, dm_2, times, rho0, t_MTO, debug=False):
    """Maps dm_1 (first memory window), tl_map until t_MTO, dm_2 after the MTO, then tl_map again."""
    n = check_tl_map_params(tl_map, rho0)
    times = np.round(times, 5)
    i_mto = int(np.where(times >= t_MTO)[0][0])
    if debug:
        print("info on piecewise application: ", i_mto, times[i_mto], len(dm_1), len(dm_2))
    i1 = min(i_mto, len(dm_1))
    if i_mto < len(dm_1):
        print("caution: t_MTO is smaller than tau_c")

    def step_map(i):
        if i < i1:
            return dm_1[i]
        if i < i_mto:
            return tl_map
        if i < i_mto + len(dm_2):
            return dm_2[i - i_mto]
        return tl_map

    return _chain(step_map, len(times), rho0.reshape(n * n), n).reshape(len(times), n, n)
