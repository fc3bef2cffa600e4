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


def get_spectrum(g1, tau, dir="", plot=False):
    """Spectrum under continuous-wave excitation from G1(tau) (correlations.py:322-380): the offset G1(tau_max) is
    subtracted, G1 is continued to negative tau as conj(G1(-tau)), and S(omega) = Re FFT, fft-shifted, on the
    energy axis 2 pi hbar fftfreq (meV). Returns (s, omega). plot=True writes the reference's three figures
    (g1_tendsymm.png, spectrum_log.png, spectrum_nolog.png) into `dir` (matplotlib; plotting is not on the
    propagation path)."""
    from ..constants import hbar
    g1 = np.array(g1, dtype=complex, copy=True)
    tau = np.asarray(tau)
    dtau = np.abs(tau[1] - tau[0])
    g1 = g1 - g1[-1]
    g1 = np.concatenate((np.conj(np.flip(g1[1:])), g1))
    tau = np.concatenate((-np.flip(tau[1:]), tau))
    s_omega = np.fft.fftshift(np.real(np.fft.fft(g1)))
    fft_freqs = np.fft.fftshift(2 * np.pi * hbar * np.fft.fftfreq(len(g1), d=dtau))
    if plot:
        import matplotlib.pyplot as plt
        for name, x, y, xl, lim in (("g1_tendsymm.png", tau, np.abs(g1), "Time (ps)", (-1, 1)),
                                    ("spectrum_log.png", fft_freqs, np.log(np.abs(s_omega)), "Frequency (meV)",
                                     (-3, 3)),
                                    ("spectrum_nolog.png", fft_freqs, np.abs(s_omega), "Frequency (meV)", (-3, 3))):
            plt.clf()
            plt.plot(x, y)
            plt.xlim(*lim)
            plt.xlabel(xl)
            plt.savefig(dir + name)
    return s_omega, fft_freqs


def _phonon_maps(system, pulses, t_mem, opA, opC, dt, rho0, options):
    """first part of the two phonon-map functions (correlations.py:876-884, 1023-1031): dynamical maps of a
    0 .. 4 t_mem run with C rho A applied at 1.2 t_mem, time-localised; the stationary map before the MTO, the
    memory-time blocks before / after it, and the last time-local map"""
    mto = {"operator": opC, "applyFrom": "_left", "applyBefore": "false", "time": 1.2 * t_mem}
    mto2 = {"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": 1.2 * t_mem}
    result, dm = system(0, 4 * t_mem, *pulses, dt=dt, rho0=rho0, multitime_op=[mto, mto2], calc_dynmap=True,
                        **options)
    _t = np.round(np.real(result[0]), 6)
    dm_tl = calc_tl_dynmap_pseudo(dm, _t)
    tl_map, dms_separated = extract_dms(dm_tl, _t, t_mem, [1.2 * t_mem])
    return tl_map, np.array(dms_separated, dtype=complex), dm_tl[-1]


def tl_three_op_two_time_phonons(system, t_axis, *pulses, t_mem=10, opA="|1><0|_2", opB="|1><1|_2",
                                 opC="|0><1|_2", tau_max=500, dt=0.1, rho0=np.array([[1, 0], [0, 0]], dtype=complex),
                                 options={"lindblad": True, "phonons": True}, debug=False, fortran_only=False):
    """<A(t) B(t + tau) C(t)> with phonons from dynamical maps (correlations.py:866-1011).

    t < t_mem: the memory-time block after the MTO comes from a dynamical-map run with the MTO at t itself; later
    t use the block of the 1.2 t_mem run; the trunk uses the block before the MTO, then the stationary map; past
    the block every row continues with the last time-local map. Same G as the reference. Its debugging side
    effects are not reproduced: the rho_test reconstruction, the figures written to pyaceqd/tests/*.png and the
    extra 0 .. 200 ps dynamical-map run at the hard-coded i_test = 9 (which makes the reference fail for fewer
    than 10 t points and for dim != 2; this one does not)."""
    if not t_axis[0] == 0:
        raise ValueError("t_axis must start at 0.")
    t_axis = np.round(t_axis, 6)
    A, B, Cm = op_to_matrix(opA), op_to_matrix(opB), op_to_matrix(opC)
    tl_map, dms_separated, tl_map2 = _phonon_maps(system, pulses, t_mem, opA, opC, dt, rho0, options)
    n_tau = int(tau_max / dt)
    tau = np.linspace(0, tau_max, n_tau + 1)
    G = np.zeros((len(t_axis), len(tau)), dtype=complex)
    dim = len(rho0[0])
    t_mem_indices = np.where(t_axis < t_mem)[0]
    dms_tauc = np.empty((len(t_mem_indices), *np.shape(dms_separated)), dtype=complex)
    for i in t_mem_indices:
        t = t_axis[i]
        mto = {"operator": opC, "applyFrom": "_left", "applyBefore": "false", "time": t}
        mto2 = {"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": t}
        result, dm = system(0, t + t_mem + 10 * dt, *pulses, dt=dt, rho0=rho0, multitime_op=[mto, mto2],
                            calc_dynmap=True, **options)
        _t = np.round(result[0], 6)
        _, _dms = extract_dms(calc_tl_dynmap_pseudo(dm, _t), _t, t_mem, [t])
        dms_tauc[i] = _dms
    n_tauc = len(dms_tauc[0, 0])
    ABC = A @ B @ Cm
    Bt = B.T.reshape(dim * dim)            # Tr(B R) = sum_ab B[b, a] R[a, b] over row-major vec(R)
    X = np.empty((dim * dim, len(t_axis)), dtype=complex)
    for i, t in enumerate(t_axis):
        rho_t = np.asarray(rho0, dtype=complex).copy().reshape(dim ** 2)
        n_steps = 0 if i == 0 else int(np.round(t / dt, 6)) + 1
        for j in range(np.min([n_steps, n_tauc]) - 1):
            rho_t = dms_separated[0, j] @ rho_t
        for j in range(n_steps - n_tauc):
            rho_t = tl_map @ rho_t
        G[i, 0] = np.trace(ABC @ rho_t.reshape(dim, dim))
        blk = dms_tauc[i, 1] if i < len(t_mem_indices) else dms_separated[1]
        for j in range(n_tauc):
            rho_t = blk[j] @ rho_t
            G[i, j + 1] = Bt @ rho_t
        X[:, i] = rho_t
    # the tails past the memory block, every row on the last time-local map, on the GPU (pqd_map_tail)
    n_tail = n_tau - n_tauc
    if n_tail > 0:
        G[:, n_tauc + 1: n_tauc + 1 + n_tail] = propagate_tau_module.map_tail(tl_map2, X, Bt, n_tail)
    return t_axis, tau, G


def tl_threeoptwotime_phonons_dm(system, t_axis, *pulses, t_mem=10, opA="|1><0|_2", opB="|1><1|_2", opC="|0><1|_2",
                                 tau_max=500, dt=0.1, rho0=np.array([[1, 0], [0, 0]], dtype=complex),
                                 options={"lindblad": True, "phonons": True}, debug=False, fortran_only=False):
    """<A(t) B(t + tau) C(t)> with phonons (correlations.py:1013-1186): for t <= t_mem the full (not time-local)
    dynamical maps E(t_k, 0) of a 0 .. t + t_mem run with the MTO at t give rho(t) = E(t, 0) rho0 and
    rho(t + tau) = E(t + tau, 0) rho0 directly; later t and every tail past the maps as in
    tl_three_op_two_time_phonons. Same G as the reference; its debugging side effects (rho_test, figures, the
    i_test = 9 run) are not reproduced."""
    if not t_axis[0] == 0:
        raise ValueError("t_axis must start at 0.")
    t_axis = np.round(t_axis, 6)
    A, B, Cm = op_to_matrix(opA), op_to_matrix(opB), op_to_matrix(opC)
    tl_map, dms_separated, tl_map2 = _phonon_maps(system, pulses, t_mem, opA, opC, dt, rho0, options)
    n_tau = int(tau_max / dt)
    tau = np.linspace(0, tau_max, n_tau + 1)
    G = np.zeros((len(t_axis), len(tau)), dtype=complex)
    dim = len(rho0[0])
    t_mem_indices = np.where(t_axis <= t_mem)[0]
    dms_tauc = []
    for i in t_mem_indices:
        t = t_axis[i]
        mto = {"operator": opC, "applyFrom": "_left", "applyBefore": "false", "time": t}
        mto2 = {"operator": opA, "applyFrom": "_right", "applyBefore": "false", "time": t}
        _, dm = system(0, t + t_mem, *pulses, dt=dt, rho0=rho0, multitime_op=[mto, mto2], calc_dynmap=True,
                       **options)
        dms_tauc.append(dm.copy())
    ABC = A @ B @ Cm
    Bt = B.T.reshape(dim * dim)
    r0 = np.asarray(rho0, dtype=complex).copy().reshape(dim ** 2)
    tails = _Tails()
    for i in range(len(t_mem_indices)):
        dm = dms_tauc[i]
        n_steps = 0 if i == 0 else int(np.round(t_axis[i] / dt, 6))
        rho_t = dm[n_steps - 1] @ r0 if n_steps > 0 else r0.copy()
        G[i, 0] = np.trace(ABC @ rho_t.reshape(dim, dim))
        rho_t_mto = rho_t.copy()
        n_map = dm.shape[0] - n_steps
        for j in range(n_map):
            rho_t_mto = dm[j + n_steps] @ r0
            G[i, j + 1] = Bt @ rho_t_mto
        tails.add(i, rho_t_mto, n_map, n_tau - n_map)
    tl_1, tl_2 = dms_separated[0], dms_separated[1]
    for i in range(len(t_mem_indices), len(t_axis)):
        rho_t = r0.copy()
        n_steps = int(np.round(t_axis[i] / dt, 6))
        for j in range(len(tl_1)):
            rho_t = tl_1[j] @ rho_t
        for j in range(n_steps - len(tl_1)):
            rho_t = tl_map @ rho_t
        G[i, 0] = np.trace(ABC @ rho_t.reshape(dim, dim))
        for j in range(tl_2.shape[0]):
            rho_t = tl_2[j] @ rho_t
            G[i, j + 1] = Bt @ rho_t
        tails.add(i, rho_t, tl_2.shape[0], n_tau - tl_2.shape[0])
    tails.run(G, tl_map2, Bt)
    return t_axis, tau, G


class _Tails:
    """The tau tails G[i, col0 + 1 + j] = Bt . tl_map2^{j+1} x_i of many rows, gathered by (col0, length) and run as
    one pqd_map_tail call per group on the GPU (one call per row paid its allocations, launch and sync
    once per t1 row)."""

    def __init__(self):
        self.groups = {}

    def add(self, i, x, col0, n):
        if n > 0:
            self.groups.setdefault((int(col0), int(n)), []).append((i, np.array(x, dtype=complex)))

    def run(self, G, tl_map2, Bt):
        for (col0, n), rows in self.groups.items():
            X = np.stack([x for _, x in rows], axis=1)
            out = propagate_tau_module.map_tail(tl_map2, X, Bt, n)
            for k, (i, _) in enumerate(rows):
                G[i, col0 + 1: col0 + 1 + n] = out[k]


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
