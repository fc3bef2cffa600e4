"""In-memory engine interface: the numeric content of an ACE param file as arrays, run on libpqd.

This is what `system_ace_stream` (general_system/general_system.py) lowers the operator strings to.
It replaces the param-file / `ACE` subprocess / outfile round trip of the reference
(pyaceqd/general_system/general_system.py:227-343) with one C-ABI call, batched over trajectories.

Objects
  System        H0, Lindblad terms, pulse channels (add_Hamiltonian / add_Lindblad / add_Pulse lines)
  Grid          ta, dt, n_steps (te = ta + n_steps dt), n_sub exponential-midpoint sub-steps
  ProcessTensor PT-MPO slices Q[s][g][d][d'], closures, dictionary map g(alpha), slice schedule
  Trajectories  per-trajectory output window [begin, end] and multi-time operators (MTOs)
"""
from dataclasses import dataclass, field
import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .constants import hbar as HBAR

KIND = {"": 0, "_left": 1, "_right": 2}


def _c(a):
    return np.ascontiguousarray(a, dtype=np.complex128)


@dataclass
class System:
    dim: int
    H0: np.ndarray
    lindblad: List[Tuple[float, np.ndarray]] = field(default_factory=list)
    channels: List[Tuple[np.ndarray, np.ndarray]] = field(default_factory=list)  # (X, samples f[k])
    sample_t0: float = 0.0
    sample_dt: float = 1.0
    hbar: float = HBAR

    def to_c(self):
        N = self.dim
        keep = {}
        keep["H0"] = _c(self.H0).reshape(N, N)
        if self.lindblad:
            keep["lr"] = np.ascontiguousarray([float(r) for r, _ in self.lindblad], dtype=np.float64)
            keep["lo"] = _c(np.stack([o for _, o in self.lindblad])).reshape(-1, N, N)
        if self.channels:
            keep["co"] = _c(np.stack([x for x, _ in self.channels])).reshape(-1, N, N)
            ns = {len(f) for _, f in self.channels}
            if len(ns) != 1:
                raise ValueError("all pulse channels must share one sample grid")
            keep["cs"] = _c(np.stack([f for _, f in self.channels]))
        s = _lib.pqd_system()
        s.dim = N
        s.hbar = float(self.hbar)
        s.H0 = _lib.cptr(keep["H0"])
        s.n_lind = len(self.lindblad)
        s.lind_rates = _lib.fptr(keep.get("lr"))
        s.lind_ops = _lib.cptr(keep.get("lo"))
        s.n_chan = len(self.channels)
        s.chan_ops = _lib.cptr(keep.get("co"))
        s.chan_samples = _lib.cptr(keep.get("cs"))
        s.n_samples = int(keep["cs"].shape[1]) if self.channels else 0
        s.sample_t0 = float(self.sample_t0)
        s.sample_dt = float(self.sample_dt)
        return s, keep


@dataclass
class Grid:
    ta: float
    dt: float
    n_steps: int
    n_sub: int = 1

    def to_c(self):
        g = _lib.pqd_grid()
        g.ta, g.dt, g.n_steps, g.n_sub = float(self.ta), float(self.dt), int(self.n_steps), int(self.n_sub)
        return g

    @property
    def times(self):
        return self.ta + self.dt * np.arange(self.n_steps + 1)


@dataclass
class ProcessTensor:
    """PT-MPO for a diagonal system-bath coupling.

    Q[s, g] is the chi x chi transfer matrix of slice s for dictionary entry g; gmap[alpha] = g for
    Liouville index alpha = i*N + j. Step n uses slice sched(n): n < n_init -> n, afterwards the
    slices [n_init, n_slices) repeat periodically (n_slices = n_init + 1: stationary / "infinite" PT).
    """
    Q: np.ndarray
    closure: np.ndarray
    closure0: np.ndarray
    bond0: np.ndarray
    gmap: np.ndarray
    n_init: int = None
    dt: Optional[float] = None
    meta: Optional[dict] = None   # generation parameters (ptgen.generation_key); stored by pt.save_pt

    def __post_init__(self):
        self.Q = _c(self.Q)
        assert self.Q.ndim == 4 and self.Q.shape[2] == self.Q.shape[3]
        self.closure = _c(self.closure).reshape(self.Q.shape[0], self.chi)
        self.closure0 = _c(self.closure0).reshape(self.chi)
        self.bond0 = _c(self.bond0).reshape(self.chi)
        self.gmap = np.ascontiguousarray(self.gmap, dtype=np.int32)
        if self.n_init is None:
            self.n_init = self.n_slices - 1
        self._handles = {}

    @property
    def chi(self):
        return self.Q.shape[2]

    @property
    def n_slices(self):
        return self.Q.shape[0]

    @property
    def D(self):
        return self.Q.shape[1]

    def schedule(self, n_steps):
        n = np.arange(n_steps, dtype=np.int64)
        per = max(1, self.n_slices - self.n_init)
        s = np.where(n < self.n_init, n, self.n_init + (n - self.n_init) % per)
        return np.ascontiguousarray(np.minimum(s, self.n_slices - 1), dtype=np.int32)

    def handle(self, ctx, dim):
        """device-resident copy (uploaded once per context, shared by all calls)"""
        key = (id(ctx), dim)
        if key not in self._handles:
            d = _lib.pqd_pt_desc()
            d.chi, d.D, d.n_slices = self.chi, self.D, self.n_slices
            d.Q, d.closure, d.closure0 = _lib.cptr(self.Q), _lib.cptr(self.closure), _lib.cptr(self.closure0)
            d.bond0, d.gmap = _lib.cptr(self.bond0), _lib.iptr(self.gmap)
            h = C.c_void_p()
            _lib.check(_lib.lib().pqd_pt_create(ctx.handle, int(dim), C.byref(d), C.byref(h)))
            self._handles[key] = (h, ctx)
        return self._handles[key][0]

    def __del__(self):
        try:
            for h, _ctx in getattr(self, "_handles", {}).values():
                _lib.lib().pqd_pt_destroy(h)
        except Exception:
            pass


@dataclass
class MTO:
    traj: int
    step: int
    before: bool
    kind: int          # 0 "", 1 "_left", 2 "_right"
    op: np.ndarray


@dataclass
class Trajectories:
    out_begin: np.ndarray
    out_end: np.ndarray
    mtos: List[MTO] = field(default_factory=list)
    system: Optional[np.ndarray] = None   # per-trajectory index into a list of systems (scans)

    @property
    def n_traj(self):
        return len(self.out_begin)

    def offsets(self, n_out):
        lens = (np.asarray(self.out_end, dtype=np.int64) - np.asarray(self.out_begin, dtype=np.int64) + 1) * n_out
        off = np.zeros(len(lens), dtype=np.int64)
        if len(lens) > 1:
            off[1:] = np.cumsum(lens)[:-1]
        return off, int(lens.sum()) if len(lens) else 0

    def to_c(self, n_out, N):
        keep = {}
        keep["b"] = np.ascontiguousarray(self.out_begin, dtype=np.int32)
        keep["e"] = np.ascontiguousarray(self.out_end, dtype=np.int32)
        off, total = self.offsets(n_out)
        keep["o"] = off
        t = _lib.pqd_traj()
        t.n_traj = self.n_traj
        t.out_begin, t.out_end, t.out_offset = _lib.iptr(keep["b"]), _lib.iptr(keep["e"]), _lib.lptr(off)
        t.n_mto = len(self.mtos)
        if self.mtos:
            keep["mt"] = np.ascontiguousarray([m.traj for m in self.mtos], dtype=np.int32)
            keep["ms"] = np.ascontiguousarray([m.step for m in self.mtos], dtype=np.int32)
            keep["mb"] = np.ascontiguousarray([1 if m.before else 0 for m in self.mtos], dtype=np.int32)
            keep["mk"] = np.ascontiguousarray([m.kind for m in self.mtos], dtype=np.int32)
            keep["mo"] = _c(np.stack([np.asarray(m.op).reshape(N, N) for m in self.mtos]))
            t.mto_traj, t.mto_step, t.mto_before = _lib.iptr(keep["mt"]), _lib.iptr(keep["ms"]), _lib.iptr(keep["mb"])
            t.mto_kind, t.mto_ops = _lib.iptr(keep["mk"]), _lib.cptr(keep["mo"])
        return t, keep, total


def split_output(out, traj, n_out):
    """flat output buffer -> list of (window_len, n_out) arrays, one per trajectory"""
    off, _ = traj.offsets(n_out)
    res = []
    for t in range(traj.n_traj):
        L = int(traj.out_end[t] - traj.out_begin[t] + 1)
        res.append(out[off[t]: off[t] + L * n_out].reshape(L, n_out))
    return res


def _systems(system):
    return list(system) if isinstance(system, (list, tuple)) else [system]


def _prep(system, grid, rho0, out_ops, traj, pt, ctx):
    systems = _systems(system)
    N = systems[0].dim
    if any(s.dim != N for s in systems):
        raise ValueError("all systems of a batch must have the same dimension")
    convs = [s.to_c() for s in systems]
    sc = (_lib.pqd_system * len(systems))(*[c for c, _ in convs])
    k1 = [k for _, k in convs]
    gc = grid.to_c()
    r0 = _c(rho0).reshape(N * N)
    ops = _c(np.stack([np.asarray(o).reshape(N, N) for o in out_ops]))
    tc, k2, total = traj.to_c(len(out_ops), N)
    pth = None
    sched = None
    if pt is not None:
        if pt.gmap.shape[0] != N * N:
            raise ValueError(f"PT gmap has {pt.gmap.shape[0]} entries, system needs {N * N}")
        if pt.dt is not None and abs(float(pt.dt) - float(grid.dt)) > 1e-9 * abs(float(grid.dt)):
            # a PT is a discretisation at its own dt (the eta_k are integrals over dt-wide slices): propagating it
            # on another grid is wrong physics, not a numerical detail
            raise ValueError(f"PT was generated for dt = {pt.dt}, the grid has dt = {grid.dt}")
        pth = pt.handle(ctx, N)
        sched = pt.schedule(max(1, grid.n_steps))
    tsys = np.ascontiguousarray(np.zeros(max(1, traj.n_traj)) if traj.system is None else traj.system, dtype=np.int32)
    if len(systems) == 1 and traj.system is not None and np.any(tsys != 0):
        raise ValueError("trajectory system index out of range")
    keep = (k1, k2, r0, ops, sched, sc, gc, tc, tsys, len(systems))
    return keep, total


def propagate(system, grid: Grid, rho0, out_ops: Sequence, traj: Trajectories,
              pt: Optional[ProcessTensor] = None, ctx=None):
    """Run all trajectories; returns a list of (window_len, n_out) complex arrays.
    `system` may be a list of Systems (parameter scan); traj.system then selects one per trajectory."""
    ctx = ctx or _lib.context()
    dim = _systems(system)[0].dim
    with ctx.lock:
        keep, total = _prep(system, grid, rho0, out_ops, traj, pt, ctx)
        k1, k2, r0, ops, sched, sc, gc, tc, tsys, n_sys = keep
        out = np.zeros(max(1, total), dtype=np.complex128)
        pth = pt.handle(ctx, dim) if pt is not None else None
        _lib.check(_lib.lib().pqd_propagate_multi(ctx.handle, n_sys, sc, _lib.iptr(tsys), C.byref(gc), pth,
                                                  _lib.iptr(sched), _lib.cptr(r0), len(out_ops), _lib.cptr(ops),
                                                  C.byref(tc), _lib.cptr(out), max(1, total)))
    return split_output(out, traj, len(out_ops))


def table_offsets(traj: Trajectories, n_out):
    """offsets of the per-trajectory ACE tables ((1 + n_out) rows of the window) in a pqd_propagate_table buffer"""
    L = np.asarray(traj.out_end, dtype=np.int64) - np.asarray(traj.out_begin, dtype=np.int64) + 1
    off = np.zeros(traj.n_traj + 1, dtype=np.int64)
    np.cumsum((1 + n_out) * L, out=off[1:])
    return off, L


def split_table(table, traj, n_out):
    """flat table buffer -> list of (1 + n_out, window_len) views, one per trajectory"""
    off, L = table_offsets(traj, n_out)
    return [table[off[t]: off[t + 1]].reshape(1 + n_out, int(L[t])) for t in range(traj.n_traj)]


def tables_from_outputs(outs, traj: Trajectories, grid: Grid):
    """host form of the device table assembly (pqd_propagate_table): per-trajectory (window_len, n_out) outputs ->
    (1 + n_out, window_len) tables with the step times in row 0 (the oracle-backed tests route through this)"""
    res = []
    for b, o in zip(traj.out_begin, outs):
        r = np.empty((1 + o.shape[1], o.shape[0]), dtype=np.complex128)
        r[0] = grid.ta + grid.dt * np.arange(int(b), int(b) + o.shape[0])
        r[1:] = o.T
        res.append(r)
    return res


def propagate_trapz(system, grid: Grid, rho0, out_ops: Sequence, traj: Trajectories, k_head, k_tail, dx,
                    pt: Optional[ProcessTensor] = None, ctx=None):
    """propagate() reduced on the device to trapezoid integrals over each trajectory's output window
    (pqd_propagate_trapz): res[t, q] = dx (y_{k_head[q]}(0) / 2 + sum_{s=1}^{L-2} y_{k_tail[q]}(s) + y_{k_tail[q]}(L-1) / 2),
    0 for windows shorter than 2 steps. The tau integrals of G2_reuse (pol_entanglement/G2.py:484-505) without
    downloading the tables. Returns (n_traj, n_pairs) complex."""
    ctx = ctx or _lib.context()
    dim = _systems(system)[0].dim
    kh = np.ascontiguousarray(k_head, dtype=np.int32)
    kt = np.ascontiguousarray(k_tail, dtype=np.int32)
    if kh.shape != kt.shape or kh.ndim != 1:
        raise ValueError("k_head and k_tail must be 1-D of equal length")
    res = np.zeros((max(1, traj.n_traj), max(1, len(kh))), dtype=np.complex128)
    with ctx.lock:
        keep, total = _prep(system, grid, rho0, out_ops, traj, pt, ctx)
        k1, k2, r0, ops, sched, sc, gc, tc, tsys, n_sys = keep
        pth = pt.handle(ctx, dim) if pt is not None else None
        _lib.check(_lib.lib().pqd_propagate_trapz(ctx.handle, n_sys, sc, _lib.iptr(tsys), C.byref(gc), pth,
                                                  _lib.iptr(sched), _lib.cptr(r0), len(out_ops), _lib.cptr(ops),
                                                  C.byref(tc), len(kh), _lib.iptr(kh), _lib.iptr(kt), float(dx),
                                                  _lib.cptr(res)))
    return res[: traj.n_traj, : len(kh)]


def propagate_table(system, grid: Grid, rho0, out_ops: Sequence, traj: Trajectories,
                    pt: Optional[ProcessTensor] = None, ctx=None):
    """propagate() returning ACE's output table per trajectory: (1 + n_out, window_len) arrays, row 0 = the step
    times grid.ta + dt * step, row 1 + k = output k (general_system.py:343), assembled on the device
    (pqd_propagate_table) so the arrays are views of one host buffer."""
    ctx = ctx or _lib.context()
    dim = _systems(system)[0].dim
    off, _ = table_offsets(traj, len(out_ops))
    n_tab = int(off[-1])
    with ctx.lock:
        keep, total = _prep(system, grid, rho0, out_ops, traj, pt, ctx)
        k1, k2, r0, ops, sched, sc, gc, tc, tsys, n_sys = keep
        table = np.empty(max(1, n_tab), dtype=np.complex128)
        pth = pt.handle(ctx, dim) if pt is not None else None
        _lib.check(_lib.lib().pqd_propagate_table(ctx.handle, n_sys, sc, _lib.iptr(tsys), C.byref(gc), pth,
                                                  _lib.iptr(sched), _lib.cptr(r0), len(out_ops), _lib.cptr(ops),
                                                  C.byref(tc), _lib.cptr(table), max(1, n_tab)))
    return split_table(table, traj, len(out_ops))


def free_propagators(system: System, grid: Grid, ctx=None):
    """M[2n + h] = free propagator of half step h of step n (N^2 x N^2, row-major vec convention)"""
    ctx = ctx or _lib.context()
    N2 = system.dim ** 2
    with ctx.lock:
        sc, keep = system.to_c()
        gc = grid.to_c()
        M = np.zeros((max(1, 2 * grid.n_steps), N2, N2), dtype=np.complex128)
        _lib.check(_lib.lib().pqd_free_propagators(ctx.handle, C.byref(sc), C.byref(gc), _lib.cptr(M)))
    return M[: 2 * grid.n_steps]


class Plan:
    """Device-resident propagation job for repeated execution (bench.py, parameter scans)."""

    def __init__(self, system, grid, rho0, out_ops, traj, pt=None, ctx=None):
        self.ctx = ctx or _lib.context()
        self.traj = traj
        self.n_out = len(out_ops)
        self.dim = _systems(system)[0].dim
        with self.ctx.lock:
            self._keep, self.total = _prep(system, grid, rho0, out_ops, traj, pt, self.ctx)
            k1, k2, r0, ops, sched, sc, gc, tc, tsys, n_sys = self._keep
            pth = pt.handle(self.ctx, self.dim) if pt is not None else None
            h = C.c_void_p()
            _lib.check(_lib.lib().pqd_plan_create_multi(self.ctx.handle, n_sys, sc, _lib.iptr(tsys), C.byref(gc),
                                                        pth, _lib.iptr(sched), _lib.cptr(r0), self.n_out,
                                                        _lib.cptr(ops), C.byref(tc), max(1, self.total),
                                                        C.byref(h)))
            self.handle = h
        self._pt = pt

    def execute(self, rebuild_free=True):
        _lib.check(_lib.lib().pqd_plan_execute(self.handle, 1 if rebuild_free else 0))

    def synchronize(self):
        """wait for the last execute; re-runs a timed-out split launch on the batched kernel, raises
        _lib.NumericError on NaN/Inf outputs"""
        _lib.check(_lib.lib().pqd_plan_synchronize(self.handle))

    PATHS = {0: "no PT (one wave per trajectory)", 1: "batched lock-step sweep", 2: "split groups",
             3: "register-resident TLS quads", 4: "split groups, several trajectories per group"}

    def info(self):
        """(path name, trajectories per workgroup, split launches that fell back to the batched kernel)"""
        p, b, f, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        _lib.check(_lib.lib().pqd_plan_info(self.handle, C.byref(p), C.byref(b), C.byref(f), C.byref(n)))
        return self.PATHS[p.value], b.value, f.value

    def windows(self):
        """True when the free propagators are built through pulse windows"""
        on = C.c_int32()
        _lib.check(_lib.lib().pqd_plan_windows(self.handle, C.byref(on)))
        return bool(on.value)

    def traj_steps(self):
        """trajectory-steps one execute propagates (shared trunks counted once per workgroup)"""
        p, b, f, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        _lib.check(_lib.lib().pqd_plan_info(self.handle, C.byref(p), C.byref(b), C.byref(f), C.byref(n)))
        return n.value

    def output_device_ptr(self):
        return _lib.lib().pqd_plan_output_device(self.handle)

    def output_tensor(self, device=None):
        """the outputs as one flat complex128 torch tensor on `device` (default: this plan's GPU), copied device to
        device after synchronize; the input of a collective gather (scan.gather_tensor)"""
        import torch
        dev = torch.device(device) if device is not None else torch.device("cuda", self.ctx.device)
        t = torch.empty(max(1, self.total), dtype=torch.complex128, device=dev)
        _lib.check(_lib.lib().pqd_plan_copy_output(self.handle, C.c_void_p(t.data_ptr()), max(1, self.total)))
        return t[: self.total]

    def download_table(self):
        """the outputs as ACE tables (propagate_table's layout): list of (1 + n_out, window_len) views"""
        n = C.c_int64()
        _lib.check(_lib.lib().pqd_plan_table_len(self.handle, C.byref(n)))
        table = np.empty(max(1, n.value), dtype=np.complex128)
        _lib.check(_lib.lib().pqd_plan_download_table(self.handle, _lib.cptr(table), max(1, n.value)))
        return split_table(table, self.traj, self.n_out)

    def download(self):
        out = np.zeros(max(1, self.total), dtype=np.complex128)
        _lib.check(_lib.lib().pqd_plan_download(self.handle, _lib.cptr(out), max(1, self.total)))
        return split_output(out, self.traj, self.n_out)

    def timing(self, reset=True):
        f, w, n = C.c_double(), C.c_double(), C.c_int32()
        _lib.check(_lib.lib().pqd_plan_timing(self.handle, C.byref(f), C.byref(w), C.byref(n), 1 if reset else 0))
        return f.value, w.value, n.value

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.lib().pqd_plan_destroy(self.handle)
                self.handle = None
        except Exception:
            pass
