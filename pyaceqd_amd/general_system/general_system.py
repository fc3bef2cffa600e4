"""system_ace_stream: pyaceqd's driver signature, lowered onto libpqd instead of the ACE binary.

Reference: pyaceqd/general_system/general_system.py:128-360. The signature is kept verbatim (plus
one optional keyword, `trajectories`, for batching) and so are the side effects callers rely on
(defaults filled into multitime_op dicts :37-42; prepare_only's return value :296). Instead of
writing a param file + pulse files, running `ACE` and parsing its outfile (:213-343), the operator
strings are evaluated to matrices (opgrammar), the pulses are sampled, and one C-ABI call
propagates every trajectory on the GPU (engine.propagate).

Engine semantics (the ACE behaviour is unobservable offline, SURVEY.md §7 "Hard parts"; each
choice is a documented switch):
  * grid t_n = t_start + n dt, n = 0..round((t_end - t_start)/dt); one output row per n (incl. t_end);
  * symmetric Trotter (use_symmetric_Trotter true, :234): M_a(n) -> PT slice -> M_b(n) per step,
    each half step an exponential-midpoint product of `n_sub` factors (default 1);
  * add_Pulse couplings X = -0.5*pi*hbar*op (:279) with the hermitian conjugate added (:245-246);
    rf channel X = -0.5*hbar*rf_op with f = omega(t) (:255);
  * pulses are sampled at spacing dt/(4 n_sub) so every midpoint is a sample (no interpolation error);
    user pulse files (`pulse_file_x/_y`, "t Re Im") are linearly interpolated and held at both ends;
  * MTO at time T acts at step round((T - t_start)/dt): applyBefore "true" before that step's
    output, otherwise after it; "" -> A rho A^dag, "_left" -> A rho, "_right" -> rho A;
  * phonons: PT from `pt_file` (pqd .npz, pyaceqd_amd.pt) or a ProcessTensor object; when no PT file exists the
    Gaussian-bath PT is generated from the same parameters as ACE's generate file (pyaceqd_amd.ptgen) and cached.
"""
import os
import warnings

import numpy as np

from ..constants import hbar
from .. import constants
from .._lib import PQDError, PQD_ERR_UNSUPPORTED
from .. import opgrammar
from ..engine import Grid, MTO, ProcessTensor, System, Trajectories, free_propagators, propagate, propagate_table, \
    propagate_trapz, KIND

temp_dir = constants.temp_dir


def sanity_checks(system_op, phonons, boson_op, initial, interaction_ops, verbose):
    """general_system.py:17-27, but raising instead of exit(1)."""
    if system_op is None and verbose:
        print("System operator not supplied, assuming TLS")
    if phonons and boson_op is None:
        raise ValueError("using phonons, but boson operator not specified")
    if initial is None and verbose:
        print("No initial state specified")
    if interaction_ops is None and verbose:
        print("No interaction hamiltonian ")


def check_multitime(multitime_op, verbose):
    """general_system.py:29-53: validate and fill defaults IN PLACE (callers rely on the mutation)."""
    if verbose:
        print("multitime operator: {}".format(multitime_op))
    if multitime_op is None:
        return
    if "operator" not in multitime_op or "time" not in multitime_op:
        raise ValueError("supply 'operator' and 'time' for multitime")
    multitime_op.setdefault("applyFrom", "")
    multitime_op.setdefault("applyBefore", "false")
    if multitime_op["applyFrom"] not in ("_left", "_right", ""):
        raise ValueError('give "_left" or "_right" or "" for multitime: {}'.format(multitime_op))


def read_result(data, n):
    """general_system.py:104-110 (kept for callers that parse ACE-format output files)."""
    t = data[:, 0]
    result = np.empty([1 + n, len(t)], dtype=complex)
    result[0] = t
    for i in range(n):
        result[i + 1] = data[:, 2 * i + 1] + 1j * data[:, 2 * i + 2]
    return result


def read_pulse_file(path):
    d = np.loadtxt(path)
    t, f = d[:, 0], d[:, 1] + 1j * d[:, 2]
    if len(t) > 1 and not np.allclose(np.diff(t), t[1] - t[0], rtol=1e-6, atol=1e-9):
        raise ValueError(f"{path}: pulse file must be uniformly sampled")
    return t, f


def generate_pulsefiles(t, pulses, temp_dir, system_prefix, suffix, abs_only=False):
    """general_system.py:55-71: write ACE-format pulse files (t Re Im, %.8f). Kept for callers that
    share one pulse file between many runs (timebin.py, pol_entanglement/G2.py)."""
    from ..tools import export_csv
    fx = temp_dir + "{}_pulse_x_{}.dat".format(system_prefix, suffix)
    fy = temp_dir + "{}_pulse_y_{}.dat".format(system_prefix, suffix)
    px, py = _sample_pulses(pulses, t, abs_only=abs_only)
    export_csv(fx, t, px.real, px.imag, precision=8, delimit=" ")
    export_csv(fy, t, py.real, py.imag, precision=8, delimit=" ")
    return fx, fy


def _ace_file_samples(t, *fs):
    """What ACE reads back from a pulse / rf file the reference writes (general_system.py:55-71, 84, 213): the
    grid np.arange(t_start, t_end, dt) and the samples, each printed with %.8f (tools.export_csv precision=8) and
    parsed again. Returns (t, f...) exactly as read_pulse_file would return them from that text."""
    q = lambda x: np.asarray(np.char.mod("%.8f", np.asarray(x, dtype=float)), dtype=float)  # noqa: E731
    return (q(t),) + tuple(q(np.real(f)) + 1j * q(np.imag(f)) for f in fs)


def _sample_pulses(pulses, t, abs_only=False):
    px = np.zeros_like(t, dtype=complex)
    py = np.zeros_like(t, dtype=complex)
    for p in pulses:
        f = p.get_total(t) * np.ones_like(t)
        if abs_only:
            f = np.abs(f)
        px = px + p.polar_x * f
        py = py + p.polar_y * f
    return px, py


def _rf_pulses(pulses):
    """generate_rf_file (:73-102): pulses re-referenced to the first pulse's start energy, chirps removed."""
    new = [p.copy() for p in pulses]
    e0, _ = new[0].get_energy()
    for p in new:
        e, _ = p.get_energy()
        p.set_energy(e - e0, 0)
    return new


def _check_pt(pt, boson_mat, dt, what):
    """A PT a run consumes must be one for this system and this grid: N^2 Liouville rows and, when
    the PT records it, the same dt (its slices integrate the bath correlations over dt-wide steps)."""
    N2 = boson_mat.shape[0] ** 2
    if pt.gmap.shape[0] != N2:
        raise ValueError(f"{what}: PT has {pt.gmap.shape[0]} Liouville rows, the system needs {N2}")
    if pt.dt is not None and abs(float(pt.dt) - float(dt)) > 1e-9 * abs(float(dt)):
        raise ValueError(f"{what}: PT was generated for dt = {pt.dt}, this run has dt = {dt}")


def _key_diff(meta, key):
    """the generation parameters in which a stored PT differs from this call's (None: none differ)"""
    if meta is None:
        return {"meta": "absent"}
    d = {k: (meta.get(k), v) for k, v in key.items() if meta.get(k) != v}
    return d or None


def _resolve_pt(pt_file, boson_mat, *, dt, t_mem, ae, temperature, threshold, factor_ah, boson_e_max, J_file,
                J_to_file, use_infinite, system_prefix, temp_dir, verbose):
    """The PT for phonons=True (general_system.py:146-211): a ProcessTensor object is used as is; an existing pqd
    PT container (`<pt_file>.npz`, or `pt_file` itself if it is one) is loaded; otherwise the Gaussian-bath PT is
    generated on the GPU from the same parameters ACE's generate file holds (pyaceqd_amd.ptgen_gpu; the host
    restatement pyaceqd_amd.ptgen with PQD_PTGEN=host) and cached under the
    reference's file name (plus `.npz`) so later calls reuse it, as the reference does with its `_initial` files.

    Provenance (VERDICT r4 missing 1 / weak 5): every PT is checked against the run (Liouville rows, dt:
    ValueError). A generated PT stores its generation parameters (ptgen.generation_key); a cached file under the
    automatic name whose parameters differ from the call's (the reference's `use_infinite` name omits a_e, t_mem and
    the bond cap) is regenerated with a warning. A file the caller named explicitly is used as given, as the reference
    uses a given pt_file, with a warning when its stored parameters differ; an explicitly named ACE file this reader
    cannot read is an error (it may hold another bath)."""
    if isinstance(pt_file, ProcessTensor):
        _check_pt(pt_file, boson_mat, dt, "pt_file")
        return pt_file
    from ..pt import load_pt, save_pt
    from .. import ptgen
    thr = float(threshold) if "e" in str(threshold).lower() or float(threshold) < 1 else 10.0 ** (-float(threshold))
    key = ptgen.generation_key(boson_mat, dt, t_mem, ae, temperature, thr, factor_ah, boson_e_max, J_file,
                               use_infinite, ptgen.default_max_bond(boson_mat))
    explicit = pt_file is not None
    if pt_file is None:
        pt_file = ptgen.pt_cache_name(system_prefix, ae, temperature, threshold, t_mem, dt, J_file=J_file,
                                      use_infinite=use_infinite)
        pt_file = os.path.join(temp_dir, pt_file) if temp_dir else pt_file
    pt_file = str(pt_file)
    from .. import ace_pt
    if ace_pt.ace_pt_exists(pt_file) and J_to_file is None:
        # ACE's own files (detected as the reference does, :153-156), read under layout ACE_PTB_V0 (ace_pt.py)
        if verbose:
            print("using pt_file " + pt_file)
        try:
            pt = ace_pt.read_ace_pt(pt_file, boson_mat.shape[0], dt=dt)
            _check_pt(pt, boson_mat, dt, pt_file + "_initial")
            return pt
        except PQDError as e:
            if e.code != PQD_ERR_UNSUPPORTED:
                raise
            if explicit:
                raise ValueError("pt_file {}_initial is not in a layout this reader knows ({}); it was named "
                                 "explicitly, so no PT is generated in its place".format(pt_file, e)) from e
            # a file in a layout other than ACE_PTB_V0 under the automatic name: the PT is taken from the pqd
            # container or generated as if no ACE file were there
            warnings.warn("{}_initial is not in a layout this reader knows ({}); using the pqd PT instead"
                          .format(pt_file, e))
    for cand in (pt_file, pt_file + ".npz"):
        if os.path.isfile(cand) and J_to_file is None:
            pt = load_pt(cand)
            _check_pt(pt, boson_mat, dt, cand)
            diff = _key_diff(pt.meta, key)
            if diff is None or (explicit and pt.meta is None):
                if verbose:
                    print("using pt_file " + cand)
                return pt
            if explicit:
                warnings.warn("pt_file {} was generated with other parameters {}; used as given".format(cand, diff))
                return pt
            warnings.warn("cached PT {} was generated with other parameters {}; regenerating".format(cand, diff))
            break
    if verbose:
        print("{} not found. Calculating...".format(pt_file))
    # generated on the GPU (ptgen_gpu: the same construction with the factorizations in csrc/ptgen.hip);
    # PQD_PTGEN=host runs the host restatement ptgen.py instead (A/B, and the CPU-only test suite)
    if os.environ.get("PQD_PTGEN", "gpu") == "host":
        gen = ptgen.qd_phonon_pt
    else:
        from .. import ptgen_gpu
        gen = ptgen_gpu.qd_phonon_pt_gpu
    pt = gen(boson_mat, dt, t_mem=t_mem, ae=ae, temperature=temperature, threshold=thr, factor_ah=factor_ah,
             boson_e_max=boson_e_max, J_file=J_file, use_infinite=use_infinite, verbose=verbose)
    try:
        save_pt(pt_file + ".npz", pt, dim=boson_mat.shape[0])
    except OSError:
        pass
    return pt


def _write_J(J_to_file, ae, factor_ah, J_file):
    """`Boson_J_print <file> 0 15 2000` (general_system.py:186-187, 203-209)."""
    from .. import ptgen
    if J_file is not None:
        J = ptgen.J_from_file(J_file)
    else:
        ah = None if factor_ah is None else ae / factor_ah
        J = lambda w: ptgen.qd_phonon_J(w, ae=ae, ah=ah)  # noqa: E731
    ptgen.write_J(J_to_file, J, 0.0, 15.0, 2000)


def system_ace_stream(t_start, t_end, *pulses, dt=0.01, phonons=False, t_mem=20.48, ae=3.0, temperature=1,
                      verbose=False, temp_dir=temp_dir, pt_file=None, suffix="", multitime_op=None,
                      pulse_file_x=None, pulse_file_y=None, system_prefix="", threshold="10", threshold_ratio="0.3",
                      buffer_blocksize="-1", dict_zero="16", precision="12", boson_e_max=7, system_op=None,
                      boson_op=None, initial=None, lindblad_ops=None, interaction_ops=None, output_ops=[],
                      prepare_only=False, LO_params=None, dressedstates=False, rf_op=None, rf_file=None,
                      firstonly=False, J_to_file=None, J_file=None, factor_ah=None, use_infinite=False,
                      print_H=False, calc_dynmap=False, rho0=None, get_M_t=None, trajectories=None, n_sub=1,
                      device=None, pulse_sampling="ace_file", trapz=None):
    """Propagate one trajectory (or a batch: `trajectories`) and return ACE's output table.

    Returns (1 + len(output_ops), n_t) complex, row 0 = time (general_system.py:104-110, 343).
    With calc_dynmap: (result, dm) with dm[i] = E(t_{i+1}, t_start) acting on row-major vec(rho)
    (general_system.py:313-336, 358-359). With `trajectories` (list of dicts with keys "multitime_op", "t_end",
    optionally "out_begin", a per-trajectory drive "pulses" / "pulse_file_x" / "pulse_file_y" and per-trajectory
    "system_op" / "lindblad_ops" replacing the call's): a list of per-trajectory results, all propagated in one launch
    (one System per distinct drive and generator: parameter scans over pulses and fields).

    pulse_sampling: "ace_file" (default, the reference's input semantics) gives the pulses the semantics of the
    files the reference hands ACE (general_system.py:55-71, 213-223): samples on np.arange(t_start, t_end, dt)
    quantised to %.8f, linearly interpolated between samples and held past t_end - dt, exactly as an explicit
    pulse_file_x/_y is read (and the rf frequency likewise, :73-84). "exact" (opt-in) samples the analytic pulses at
    dt/(4 n_sub) instead, so every exponential midpoint is a sample of the analytic field. The two differ by
    O(dt^2 f'') (about 1e-4 relative for tau_0 = 3 ps at dt = 0.1), above the no-phonon 1e-8 tolerance, which is
    why the drop-in default is the reference's.
    """
    if pulse_sampling not in ("exact", "ace_file"):
        raise ValueError(f"pulse_sampling must be 'exact' or 'ace_file', not {pulse_sampling!r}")
    sanity_checks(system_op, phonons, boson_op, initial, interaction_ops, verbose)
    if multitime_op is not None:
        if isinstance(multitime_op, dict):
            multitime_op = [multitime_op]
        for m in multitime_op:
            check_multitime(m, verbose)
    if phonons and J_to_file:
        _write_J(J_to_file, ae, factor_ah, J_file)
    if prepare_only:
        return [np.array([0, 0]) for _ in range(1 + len(output_ops))]
    if dressedstates or print_H:
        raise NotImplementedError("dressed-state / print_H diagnostics are out of scope (SURVEY.md §2)")
    if LO_params is not None:
        raise NotImplementedError("add_single_mode (LO phonons) is out of scope (SURVEY.md §2)")

    # ---------------------------------------------------------------- operators
    dim = None
    for s in ([initial] if initial else []) + list(output_ops) + [op for op, _ in (interaction_ops or [])] \
            + list(system_op or []):
        v = opgrammar.evaluate(s)
        if isinstance(v, np.ndarray):
            dim = v.shape[0]
            break
    if dim is None:
        dim = 2  # "assuming TLS" (:19)
    mat = lambda s: opgrammar.to_matrix(s, dim)  # noqa: E731
    def hamiltonian(ops):
        H = np.zeros((dim, dim), dtype=complex)
        for s in (ops or []):
            H = H + mat(s)
        return H

    def dissipators(ops):
        return [(float(rate), mat(op)) for op, rate in (ops or [])]
    rho_init = mat(initial) if initial is not None else np.diag([1.0] + [0.0] * (dim - 1)).astype(complex)
    if rho0 is not None:
        rho_init = np.asarray(rho0, dtype=complex).reshape(dim, dim)

    # ---------------------------------------------------------------- time grid(s)
    n_steps = int(round((t_end - t_start) / dt))
    traj_specs = trajectories if trajectories is not None else [{"multitime_op": multitime_op, "t_end": t_end}]
    traj_steps = []
    for spec in traj_specs:
        te = spec.get("t_end", t_end)
        traj_steps.append(int(round((te - t_start) / dt)))
        mt = spec.get("multitime_op")
        if isinstance(mt, dict):
            spec["multitime_op"] = [mt]
        for m in spec.get("multitime_op") or []:
            check_multitime(m, verbose)
    n_steps = max([n_steps] + traj_steps) if trajectories is not None else n_steps
    grid = Grid(t_start, dt, n_steps, n_sub)

    # ---------------------------------------------------------------- pulse channels
    ds = dt / (4 * n_sub)
    ts = t_start + ds * np.arange(4 * n_sub * n_steps + 1)
    # the reference's pulse-file grid (:213); a batch shares one file per drive, up to its longest trajectory
    t_file = np.arange(t_start, t_start + n_steps * dt if trajectories is not None else t_end, step=dt / 1)

    def make_system(pulse_list, pfx, pfy, H0, lind):
        channels, t0s, dts = [], [], []
        use_pulses = [pulse_list[0]] if (firstonly and pulse_list) else list(pulse_list)
        if rf_op is not None and rf_file is None:
            use_pulses = _rf_pulses(use_pulses)

        def add_channel(op_str, scale, t_s, f):
            channels.append((scale * mat(op_str), np.asarray(f, dtype=complex)))
            t0s.append(t_s[0])
            dts.append(t_s[1] - t_s[0] if len(t_s) > 1 else ds)

        if interaction_ops:
            fx = fy = None
            tx = ty = ts
            if pfx is not None:
                tx, fx = read_pulse_file(pfx)
            if pfy is not None:
                ty, fy = read_pulse_file(pfy)
            if fx is None or fy is None:
                if pulse_sampling == "ace_file":
                    tf, sx, sy = _ace_file_samples(t_file, *_sample_pulses(use_pulses, t_file))
                    if fx is None:
                        tx = tf
                    if fy is None:
                        ty = tf
                else:
                    sx, sy = _sample_pulses(use_pulses, ts)
                if fx is None:
                    fx = sx
                if fy is None:
                    fy = sy
            for op, pol in interaction_ops:
                if pol == "y":
                    add_channel(op, -0.5 * np.pi * hbar, ty, fy)
                else:
                    add_channel(op, -0.5 * np.pi * hbar, tx, fx)
        if rf_op is not None:
            if rf_file is not None:
                tr, fr = read_pulse_file(rf_file)
            elif pulse_sampling == "ace_file":
                tr, fr = _ace_file_samples(t_file, np.asarray(pulse_list[0].get_frequency(t_file), dtype=complex)
                                           * np.ones_like(t_file))
            else:
                tr, fr = ts, np.asarray(pulse_list[0].get_frequency(ts), dtype=complex) * np.ones_like(ts)
            add_channel(rf_op, -0.5 * hbar, tr, fr)
        # all channels must share one sample grid: resample onto the finest common raster if needed
        if channels and (len(set(np.round(t0s, 12))) > 1 or len(set(np.round(dts, 12))) > 1
                         or len({len(f) for _, f in channels}) > 1):
            res = []
            for (X, f), t0c, dtc in zip(channels, t0s, dts):
                tc = t0c + dtc * np.arange(len(f))
                res.append((X, np.interp(ts, tc, f.real) + 1j * np.interp(ts, tc, f.imag)))
            channels = res
            t0s, dts = [ts[0]], [ds]
        return System(dim=dim, H0=H0, lindblad=lind, channels=channels,
                      sample_t0=t0s[0] if channels else 0.0, sample_dt=dts[0] if channels else 1.0)

    # per-trajectory drive (scans): a spec may carry its own "pulses" / "pulse_file_x" / "pulse_file_y"; every
    # distinct drive becomes one System of a multi-system launch (engine.propagate, traj.system)
    sys_keys, systems, traj_sys = {}, [], []
    for spec in traj_specs:
        pl = tuple(spec["pulses"]) if "pulses" in spec else tuple(pulses)
        pfx = spec.get("pulse_file_x", pulse_file_x)
        pfy = spec.get("pulse_file_y", pulse_file_y)
        sop = spec.get("system_op", system_op)
        lop = spec.get("lindblad_ops", lindblad_ops)
        key = (tuple(id(p) for p in pl), pfx, pfy, tuple(sop or ()), tuple((str(o), float(r)) for o, r in (lop or ())))
        if key not in sys_keys:
            sys_keys[key] = len(systems)
            systems.append(make_system(pl, pfx, pfy, hamiltonian(sop), dissipators(lop)))
        traj_sys.append(sys_keys[key])
    system = systems[0]

    if get_M_t is not None:
        g1 = Grid(get_M_t, dt, 1, n_sub)
        M = free_propagators(system, g1)
        return M[1] @ M[0]

    # ---------------------------------------------------------------- environment
    pt = None
    if phonons:
        pt = _resolve_pt(pt_file, mat(boson_op), dt=dt, t_mem=t_mem, ae=ae, temperature=temperature,
                         threshold=threshold, factor_ah=factor_ah, boson_e_max=boson_e_max, J_file=J_file,
                         J_to_file=J_to_file, use_infinite=use_infinite, system_prefix=system_prefix,
                         temp_dir=temp_dir, verbose=verbose)

    # ---------------------------------------------------------------- trajectories
    out_mats = [mat(s) for s in output_ops]
    if calc_dynmap:
        return _dynmap(system, grid, pt, rho_init, multitime_op, out_mats, t_start, dt, dim, device)
    begins, ends, mtos = [], [], []
    for k, spec in enumerate(traj_specs):
        e = traj_steps[k] if trajectories is not None else n_steps
        b = spec.get("out_begin", 0)
        begins.append(b)
        ends.append(e)
        for m in spec.get("multitime_op") or []:
            mtos.append(_mto(k, m, t_start, dt, mat))
    if not out_mats:
        out_mats = [np.eye(dim, dtype=complex)]
        n_real = 0
    else:
        n_real = len(out_mats)
    multi = len(systems) > 1
    tr = Trajectories(np.array(begins), np.array(ends), mtos, system=np.array(traj_sys) if multi else None)
    from .. import _lib
    if trapz is not None:
        # (k_head, k_tail, dx): per-trajectory trapezoid integrals of output rows over the window, on the device
        # (pqd_propagate_trapz), in place of the tables: (n_traj, n_pairs) complex
        if not n_real:
            raise ValueError("trapz needs output_ops")
        k_head, k_tail, dx = trapz
        res = propagate_trapz(systems if multi else system, grid, rho_init, out_mats, tr, k_head, k_tail, dx, pt=pt,
                              ctx=_lib.context(device))
        return res if trajectories is not None else res[0]
    if n_real:
        # ACE's output table per trajectory, assembled on the device (pqd_propagate_table): views, no host copies
        res = propagate_table(systems if multi else system, grid, rho_init, out_mats, tr, pt=pt,
                              ctx=_lib.context(device))
        return res if trajectories is not None else res[0]
    outs = propagate(systems if multi else system, grid, rho_init, out_mats, tr, pt=pt, ctx=_lib.context(device))
    results = []
    for k, o in enumerate(outs):
        steps = np.arange(begins[k], ends[k] + 1)
        r = np.empty((1 + n_real, len(steps)), dtype=complex)
        r[0] = t_start + dt * steps
        if n_real:
            r[1:] = o.T
        results.append(r)
    return results if trajectories is not None else results[0]


def _mto(traj, m, t_start, dt, mat):
    step = int(round((float(m["time"]) - t_start) / dt))
    before = str(m.get("applyBefore", "false")).lower() == "true"
    return MTO(traj=traj, step=step, before=before, kind=KIND[m.get("applyFrom", "")], op=mat(m["operator"]))


def _dynmap(system, grid, pt, rho_init, multitime_op, out_mats, t_start, dt, dim, device):
    """dm[i] = E(t_{i+1}, t_start): N^2 trajectories, trajectory beta starts from the basis element |i><j|
    (prepared from |0><0| by two MTOs at step 0), outputs all matrix elements."""
    from .. import _lib
    N = dim
    N2 = N * N
    ket = lambda a, b: np.outer(np.eye(N)[a], np.eye(N)[b]).astype(complex)  # noqa: E731
    ops = [ket(a % N, a // N) for a in range(N2)]  # <|j><i|> = rho[i][j]  for alpha = i*N + j
    mtos = []
    for beta in range(N2):
        i, j = divmod(beta, N)
        mtos.append(MTO(beta, 0, True, 1, ket(i, 0)))
        mtos.append(MTO(beta, 0, True, 2, ket(0, j)))
        for m in multitime_op or []:
            mtos.append(_mto(beta, m, t_start, dt, lambda s: opgrammar.to_matrix(s, dim)))
    tr = Trajectories(np.zeros(N2, dtype=int), np.full(N2, grid.n_steps), mtos)
    outs = propagate(system, grid, ket(0, 0), ops, tr, pt=pt, ctx=_lib.context(device))
    E = np.stack(outs, axis=2)                      # (n_t, alpha, beta)
    dm = E[1:]
    # regular result from rho_init
    rho_vec = np.asarray(rho_init, dtype=complex).reshape(N2)
    rhos = E @ rho_vec                               # (n_t, N2)
    res = np.empty((1 + len(out_mats), grid.n_steps + 1), dtype=complex)
    res[0] = grid.times
    for k, O in enumerate(out_mats):
        res[1 + k] = np.einsum("ij,nji->n", O, rhos.reshape(-1, N, N))
    return res, dm
