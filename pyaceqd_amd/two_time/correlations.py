"""One- and two-time correlation drivers (pyaceqd/two_time/correlations.py), on libpqd.

The reference runs one ACE process per t1 point on a ThreadPoolExecutor (`_ops_two_time`,
correlations.py:135-184), each re-propagating the shared trunk 0 -> t1. Here every t1 point is one
trajectory of a single batched launch (system_ace_stream(..., trajectories=[...])): the GPU
propagates all of them in lock-step, each trajectory only stores the last n_tau+1 output rows the
caller slices out (`G[j,1:] = out_B[-n_tau:]`, `G[j,0] = out_ABC[-(n_tau+1)]`, :181-183).
Function names, signatures, option-dict side effects and return values are the reference's.
The dynamical-map variants (tl_*) call the GPU map-chain sweep (propagate_tau_module).
"""
import numpy as np

from ..tools import calc_tl_dynmap_pseudo, extract_dms, op_to_matrix, tl_pad_stationary_nsteps
from ..two_level_system.tls import tls  # noqa: F401  (reference default system)
from . import propagate_tau_module


def _ops_one_time(system, *pulses, t0=-500, t_MTO=0, tend=500, dt=0.1, options={"lindblad": True, "phonons": False},
                  debug=False):
    t, out_b, out_0 = system(t0, tend, *pulses, dt=dt, **options)
    t = np.round(t, 6)
    n_tau = int((tend - t_MTO) / dt) + 1
    tau = np.linspace(t_MTO, tend, n_tau)
    G = np.empty(n_tau, dtype=complex)
    i = int(np.where(t == t_MTO)[0][0])
    G[0] = out_0[i]
    G[1:] = out_b[i + 1:]
    return tau, G


def two_op_one_time(system, *pulses, opA="|1><0|_2", opB="|0><1|_2", t0=-500, t_MTO=0, tend=500, dt=0.1,
                    options={"lindblad": True, "phonons": False}, debug=False):
    """<A(t_MTO + tau) B(t_MTO)>   (correlations.py:54-91)"""
    options["output_ops"] = [opA, "(" + opA + "*" + opB + ")"]
    options["multitime_op"] = [{"operator": opB, "applyFrom": "_left", "applyBefore": "false", "time": t_MTO}]
    return _ops_one_time(system, *pulses, t0=t0, t_MTO=t_MTO, tend=tend, dt=dt, options=options, debug=debug)


def three_op_one_time(system, *pulses, opA="|1><0|_2", opB="|1><1|_2", opC="|0><1|_2", t0=-500, t_MTO=0, tend=500,
                      dt=0.1, options={"lindblad": True, "phonons": False}, debug=False):
    """<A(t_MTO) B(t_MTO + tau) C(t_MTO)>   (correlations.py:93-133)"""
    options["output_ops"] = [opB, "(" + opA + "*" + opB + "*" + opC + ")"]
    options["multitime_op"] = [{"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": t_MTO},
                               {"operator": opC, "applyFrom": "_left", "applyBefore": "false", "time": t_MTO}]
    return _ops_one_time(system, *pulses, t0=t0, t_MTO=t_MTO, tend=tend, dt=dt, options=options, debug=debug)


def _ops_two_time(system, t_axis, *pulses, mtos=[], tau_max=500, dt=0.1, options={"lindblad": True, "phonons": False},
                  debug=False, workers=15, n_mto=None, t_start=0):
    """Batched replacement of the per-t1 ACE fan-out (correlations.py:135-184). `workers` is accepted for
    signature compatibility; all t1 trajectories run in one GPU launch."""
    if n_mto is None or len(mtos) < n_mto:
        raise ValueError("multi-time operators are required for the two-time correlation function.")
    if t_start > 0:
        raise ValueError("t_start > 0 is not supported yet. Use t_start<=0 to e.g. reach a stationary state "
                         "before applying the MTO.")
    extra = [dict(m) for m in mtos[n_mto:]]
    t1 = np.asarray(t_axis)
    n_tau = int(tau_max / dt)
    tau = np.linspace(0, tau_max, n_tau + 1)
    specs = []
    for t1_i in t1:
        tend = t1_i + tau_max
        ms = []
        for j in range(n_mto):
            m = dict(mtos[j])
            m["time"] = t1_i
            ms.append(m)
        ms += [dict(m) for m in extra]
        n_i = int(round((tend - t_start) / dt))
        specs.append({"multitime_op": ms, "t_end": tend, "out_begin": max(0, n_i - n_tau)})
    tend_max = float(np.max(t1)) + tau_max if len(t1) else tau_max
    results = system(t_start, tend_max, *pulses, dt=dt, trajectories=specs, **options)
    G = np.empty((len(t1), len(tau)), dtype=complex)
    for j, r in enumerate(results):
        G[j, 1:] = r[1][-n_tau:]
        G[j, 0] = r[2][-(n_tau + 1)]
    return t1, tau, G


def two_op_two_time(system, t_axis, *pulses, opA="|1><0|_2", opB="|0><1|_2", tau_max=500, dt=0.1,
                    options={"lindblad": True, "phonons": False}, debug=False, workers=15):
    """<A(t + tau) B(t)>, e.g. G1(t, tau)   (correlations.py:186-225)"""
    options["output_ops"] = [opA, "(" + opA + "*" + opB + ")"]
    mtos = [{"operator": opB, "applyFrom": "_left", "applyBefore": "false"}]
    return _ops_two_time(system, t_axis, *pulses, mtos=mtos, tau_max=tau_max, dt=dt, options=options, debug=debug,
                         workers=workers, n_mto=1)


def three_op_two_time(system, t_axis, *pulses, opA="|1><0|_2", opB="|1><1|_2", opC="|0><1|_2", tau_max=500, dt=0.1,
                      t_start=0, options={"lindblad": True, "phonons": False}, debug=False, workers=15):
    """<A(t) B(t + tau) C(t)>, e.g. G2(t, tau)   (correlations.py:227-270)"""
    options["output_ops"] = [opB, "(" + opA + "*" + opB + "*" + opC + ")"]
    mtos = [{"operator": opA, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": opC, "applyFrom": "_left", "applyBefore": "false"}]
    return _ops_two_time(system, t_axis, *pulses, mtos=mtos, tau_max=tau_max, dt=dt, options=options, debug=debug,
                         workers=workers, n_mto=2, t_start=t_start)


def five_op_two_time(system, t_axis, *pulses, opA="|1><0|_2", opB="|1><0|_2", opC="|1><1|_2", opD="|0><1|_2",
                     opE="|0><1|_2", tau_max=500, dt=0.1, t_start=-500, options={"lindblad": True, "phonons": False},
                     debug=False, workers=15):
    """<A(0) B(t) C(t + tau) D(t) E(0)>   (correlations.py:272-320; same tau=0 caveat as the reference)"""
    options["output_ops"] = [opC, "(" + opA + "*" + opB + "*" + opC + "*" + opD + "*" + opE + ")"]
    mtos = [{"operator": opB, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": opD, "applyFrom": "_left", "applyBefore": "false"},
            {"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": 0},
            {"operator": opE, "applyFrom": "_left", "applyBefore": "false", "time": 0}]
    return _ops_two_time(system, t_axis, *pulses, mtos=mtos, tau_max=tau_max, dt=dt, options=options, debug=debug,
                         workers=workers, n_mto=2, t_start=t_start)


def _tl_sweep(system, t_axis, pulses, t_mem, ops, tau_max, dt, rho0, options, use_dm, fortran_only, mtos_dyn,
              stationary_ops):
    """Shared body of tl_two_op_two_time / tl_three_op_two_time (correlations.py:450-615, 696-863).

    ops = (A, B, C): G(t, 0) = Tr(A B C rho(t)), rho -> C rho A at t, G(t, tau) = Tr(B rho(t + tau)).
    use_dm, fortran_only=True  -> the reference's Fortran call (:781-782): calc_onetime_parallel on the GPU, which
                                  reads the row-major vec(rho) column-major (it works with rho^T);
    use_dm, fortran_only=False -> the reference's row-major Python loop (:786-838: trunk `while _t[j] < t`,
                                  Tr(ABC rho), C rho A, propagate_tau from map j, Tr(B rho_tau)). The same
                                  calc_onetime_parallel kernel computes it exactly when handed (C^T, B^T, A^T): the
                                  column-major view of vec(R) is R^T, Tr(C^T B^T A^T R^T) = Tr(A B C R), the MTO gives
                                  A^T R^T C^T = (C R A)^T and Tr(B^T X^T) = Tr(B X). One launch for all t instead of one
                                  propagate_tau per t.
    not use_dm                 -> the stationary time-local map of a 0 .. 4 t_mem dynamical-map run with the MTOs at
                                  2 t_mem (:743-750, :840-860), with `stationary_ops` = (A', B') giving
                                  G(t, 0) = Tr(A' B' rho), rho -> B' rho, G(t, tau) = Tr(A' rho_tau) as the reference
                                  writes it (for the three-op function that is its two-op formula, :856-860).
    """
    if not t_axis[0] == 0:
        raise ValueError("t_axis must start at 0.")
    opA_mat, opB_mat, opC_mat = ops
    dim = len(rho0[0])
    n_tau = int(tau_max / dt)
    tau = np.linspace(0, tau_max, n_tau + 1)
    if use_dm:
        tend = t_axis[-1] + tau_max
        result, dm = system(0, tend, *pulses, dt=dt, rho0=rho0, multitime_op=[], calc_dynmap=True, **options)
        _t = np.round(np.real(result[0]), 6)
        dm_tl = calc_tl_dynmap_pseudo(dm, _t)
        dm_tl_f = np.asfortranarray(dm_tl.transpose(1, 2, 0))
        if fortran_only:
            a, b, c = opA_mat, opB_mat, opC_mat
        else:
            a, b, c = opC_mat.T, opB_mat.T, opA_mat.T
        G = propagate_tau_module.calc_onetime_parallel(dm_tl_f, np.asarray(rho0).reshape(dim ** 2), n_tau, dim, a, b,
                                                       c, _t, t_axis)
        return t_axis, tau, np.ascontiguousarray(G)
    result, dm = system(0, 4 * t_mem, *pulses, dt=dt, rho0=rho0, multitime_op=mtos_dyn, calc_dynmap=True, **options)
    _t = np.round(np.real(result[0]), 6)
    dm_tl = calc_tl_dynmap_pseudo(dm, _t)
    tl_map, _ = extract_dms(dm_tl, _t, t_mem, [2 * t_mem])
    G = np.zeros((len(t_axis), len(tau)), dtype=complex)
    if options.get("phonons", False):
        print("phonons not implemented yet")
        return t_axis, tau, G
    sA, sB = stationary_ops
    rho_t = np.asarray(rho0, dtype=complex).copy().reshape(dim ** 2)
    for i, t in enumerate(t_axis):
        n_steps = 0 if i == 0 else int((t - t_axis[i - 1]) / dt)
        rho_t = np.linalg.matrix_power(tl_map, n_steps) @ rho_t
        R = rho_t.reshape(dim, dim)
        G[i, 0] = np.trace(sA @ sB @ R)
        rho_tau = tl_pad_stationary_nsteps(tl_map, n_tau, sB @ R)
        G[i, 1:] = np.trace(sA @ rho_tau, axis1=1, axis2=2)
    return t_axis, tau, G


def tl_two_op_two_time(system, t_axis, *pulses, t_mem=10, opA="|1><0|_2", opB="|0><1|_2", tau_max=500, dt=0.1,
                       rho0=np.array([[1, 0], [0, 0]], dtype=complex), options={"lindblad": True, "phonons": False},
                       debug=False, workers=15, use_dm=False, fortran_only=False):
    """<A(t + tau) B(t)> from dynamical maps (correlations.py:450-615; use_dm -> GPU map-chain sweep, either
    convention of `fortran_only`)"""
    A, B = op_to_matrix(opA), op_to_matrix(opB)
    I = np.identity(A.shape[0], dtype=complex)
    mto = {"operator": opB, "applyFrom": "_left", "applyBefore": "false", "time": 2 * t_mem}
    # <A(t+tau) B(t)> = Tr(A E(tau) [B rho(t)]): the reference passes (identity, A, B) as (opA, opB, opC) (:534)
    return _tl_sweep(system, t_axis, pulses, t_mem, (I, A, B), tau_max, dt, rho0, options, use_dm, fortran_only,
                     [mto], (A, B))


def tl_three_op_two_time(system, t_axis, *pulses, t_mem=10, opA="|1><0|_2", opB="|1><1|_2", opC="|0><1|_2",
                         tau_max=500, dt=0.1, rho0=np.array([[1, 0], [0, 0]], dtype=complex),
                         options={"lindblad": True, "phonons": False}, debug=False, workers=15, use_dm=False,
                         fortran_only=False, three_op_stationary=False):
    """<A(t) B(t + tau) C(t)> from dynamical maps (correlations.py:696-863).

    Without use_dm the reference evaluates its TWO-op formula here, ignoring opC: G(t, 0) = Tr(A B rho),
    rho -> B rho, G(t, tau) = Tr(A rho_tau) (:856-860); that is reproduced by default (pinned by
    tests/golden/pyref_correlations.npz). `three_op_stationary=True` (not in the reference) evaluates the three-op
    correlation on the stationary map instead: Tr(A B C rho), rho -> C rho A, Tr(B rho_tau)."""
    A, B, Cm = op_to_matrix(opA), op_to_matrix(opB), op_to_matrix(opC)
    mto = {"operator": opC, "applyFrom": "_left", "applyBefore": "false", "time": 2 * t_mem}
    mto2 = {"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": 2 * t_mem}
    if three_op_stationary:
        if use_dm:
            raise ValueError("three_op_stationary applies to the stationary-map branch (use_dm=False) only")
        return _tl_stationary_three_op(system, t_axis, pulses, t_mem, (A, B, Cm), tau_max, dt, rho0, options,
                                       [mto, mto2])
    return _tl_sweep(system, t_axis, pulses, t_mem, (A, B, Cm), tau_max, dt, rho0, options, use_dm, fortran_only,
                     [mto, mto2], (A, B))


def _tl_stationary_three_op(system, t_axis, pulses, t_mem, ops, tau_max, dt, rho0, options, mtos_dyn):
    """opt-in three-op form of the stationary-map branch (see tl_three_op_two_time)"""
    A, B, Cm = ops
    dim = len(rho0[0])
    n_tau = int(tau_max / dt)
    tau = np.linspace(0, tau_max, n_tau + 1)
    result, dm = system(0, 4 * t_mem, *pulses, dt=dt, rho0=rho0, multitime_op=mtos_dyn, calc_dynmap=True, **options)
    _t = np.round(np.real(result[0]), 6)
    tl_map, _ = extract_dms(calc_tl_dynmap_pseudo(dm, _t), _t, t_mem, [2 * t_mem])
    G = np.zeros((len(t_axis), len(tau)), dtype=complex)
    rho_t = np.asarray(rho0, dtype=complex).copy().reshape(dim ** 2)
    for i, t in enumerate(t_axis):
        n_steps = 0 if i == 0 else int((t - t_axis[i - 1]) / dt)
        rho_t = np.linalg.matrix_power(tl_map, n_steps) @ rho_t
        R = rho_t.reshape(dim, dim)
        G[i, 0] = np.trace(A @ B @ Cm @ R)
        rho_tau = tl_pad_stationary_nsteps(tl_map, n_tau, Cm @ R @ A)
        G[i, 1:] = np.trace(B @ rho_tau, axis1=1, axis2=2)
    return t_axis, tau, G
