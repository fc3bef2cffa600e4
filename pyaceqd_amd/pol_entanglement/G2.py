"""Polarisation-entanglement tomography (pyaceqd/pol_entanglement/G2.py:11-606), on libpqd.

Same class, constructor and methods as the reference `PolarizatzionEntanglement`. The reference fans the t1 grid
out over a ThreadPoolExecutor, one ACE process per t1 point (G1 :186-201, G2 :243-258, G2_reuse :467-482). Here
every t1 point is one trajectory of a single batched `system(..., trajectories=[...])` call: one GPU launch per
G1 / G2 / G2_reuse, all t1 trajectories in lock step. `workers` is accepted and ignored. Each trajectory's output
window starts where the reference starts slicing it (`int(t1/dt)` for G2, the last n_tau+1 rows for G1), so the
per-t1 arrays are the reference's slices.

Everything after the propagation (tau/t integrals, the 4x4 two-photon density matrix, concurrence, spectra) is
host post-processing and follows the reference's formulas; the nested integrals of `integrate_timedep_G2` are
evaluated with cumulative trapezoids instead of re-integrating every (t, t') pair.
"""
import os

import numpy as np

from .. import constants
from ..constants import hbar
from ..tools import concurrence, construct_t, export_csv, simple_t_gaussian

temp_dir = constants.temp_dir


def _trapz(y, x, axis=-1):
    return np.trapezoid(y, x, axis=axis)


class PolarizatzionEntanglement():
    def __init__(self, system, sigma_x, sigma_y, sigma_xdag, sigma_ydag, *pulses, dt=0.1, tend=400,
                 time_intervals=None, simple_exp=True, dt_small=0.1, gaussian_t=None, regular_grid=False,
                 verbose=False, workers=2, remove_files=True, factor_tau=4, options={}) -> None:
        """See pyaceqd/pol_entanglement/G2.py:12-103 for the parameters; `workers` is unused (one batched launch)."""
        self.system = system
        self.dt = dt
        self.options = dict(options)
        self.options["dt"] = dt
        self.tend = tend
        self.remove_files = remove_files
        self.simple_exp = simple_exp
        self.gaussian_t = gaussian_t
        self.pulses = pulses
        self.workers = workers
        self.ax = "(" + sigma_x + ")"
        self.ay = "(" + sigma_y + ")"
        self.axdag = "(" + sigma_xdag + ")"
        self.aydag = "(" + sigma_ydag + ")"
        if "temp_dir" in options:
            self.temp_dir = options["temp_dir"]
        else:
            print("temp_dir not included in options, setting to temp_dir specified in constants")
            self.options["temp_dir"] = temp_dir
            self.temp_dir = temp_dir
        given = "pulse_file_x" in self.options or ("pulse_file_y" in self.options
                                                   and self.options["pulse_file_x"] is not None
                                                   and self.options["pulse_file_y"] is not None)
        self._own_files = False
        if given:
            self.remove_files = False
        else:
            self.prepare_pulsefile(verbose=verbose)
            self.options["pulse_file_x"] = self.pulse_file_x
            self.options["pulse_file_y"] = self.pulse_file_y
            self._own_files = True
        self.gamma_e = options["gamma_e"]
        if regular_grid:
            self.t1 = np.arange(0, self.tend + dt_small, dt_small)
        elif time_intervals is not None:
            if len(time_intervals) != 2:
                return ValueError("time_intervals must be a list of length 2")  # sic (reference :86-87)
            a, b = time_intervals
            self.t1 = np.concatenate([np.arange(0, a, dt_small), np.arange(a, b, 10 * dt_small),
                                      np.round(np.exp(np.arange(np.log(b), np.log(tend), dt_small))),
                                      np.array([tend])])
        elif self.gaussian_t is not None:
            self.t1 = simple_t_gaussian(0, self.gaussian_t, self.tend, dt_small, 10 * dt_small, *self.pulses,
                                        decimals=1, exp_part=self.simple_exp)
        else:
            self.t1 = construct_t(0, self.tend, dt_small, 1 * dt_small, dt_small, *self.pulses,
                                  simple_exp=self.simple_exp, factor_tau=factor_tau)

    def prepare_pulsefile(self, verbose=False):
        """x/y pulse files on [0, tend) at dt/5, 8 decimals (reference :105-118)"""
        ts = np.arange(0, self.tend, step=self.dt / 5)
        self.pulse_file_x = self.temp_dir + "polar_ent_pulse_x_{}.dat".format(id(self))
        self.pulse_file_y = self.temp_dir + "polar_ent_pulse_y_{}.dat".format(id(self))
        px = np.zeros_like(ts, dtype=complex)
        py = np.zeros_like(ts, dtype=complex)
        for p in self.pulses:
            f = p.get_total(ts)
            px = px + p.polar_x * f
            py = py + p.polar_y * f
        export_csv(self.pulse_file_x, ts, px.real, px.imag, precision=8, delimit=" ", verbose=verbose)
        export_csv(self.pulse_file_y, ts, py.real, py.imag, precision=8, delimit=" ", verbose=verbose)

    def __del__(self):
        if getattr(self, "remove_files", False) and getattr(self, "_own_files", False):
            for f in (self.pulse_file_x, self.pulse_file_y):
                try:
                    os.remove(f)
                except OSError:
                    pass

    # ------------------------------------------------------------------ batched propagation
    def _batch(self, t_end_of, out_begin_of, mtos_of, output_ops, t_end_max):
        specs = [{"multitime_op": mtos_of(i), "t_end": t_end_of(i), "out_begin": out_begin_of(i)}
                 for i in range(len(self.t1))]
        opts = dict(self.options)
        opts["output_ops"] = output_ops
        return self.system(0, t_end_max, trajectories=specs, **opts)

    def _g2_specs(self, op1_t, op23s, op4_t):
        """one trajectory per t1 (reference :467-482): op4 from the left and op1 from the right at t1, every
        trajectory to tend, its outputs from step int(t1/dt) on; output operators <op2 op3> for every pair, then
        <op1 op2 op3 op4>"""
        tau0 = [op1_t + " * " + o + " * " + op4_t for o in op23s]
        specs = [{"multitime_op": [{"operator": op1_t, "applyFrom": "_right", "applyBefore": "false", "time": t},
                                   {"operator": op4_t, "applyFrom": "_left", "applyBefore": "false", "time": t}],
                  "t_end": self.tend, "out_begin": max(0, int(t / self.dt))} for t in self.t1]
        return specs, list(op23s) + tau0, int(self.tend / self.dt)

    def _g2_runs(self, op1_t, op23s, op4_t):
        """per-t1 arrays (1 + 2 n_pairs, n_t2 + 1) starting at step int(t1/dt), one launch"""
        specs, outs, n_tau = self._g2_specs(op1_t, op23s, op4_t)
        opts = dict(self.options)
        opts["output_ops"] = outs
        return n_tau, self.system(0, self.tend, trajectories=specs, **opts)

    def _reuse_integrals(self, res, n_pairs, n_tau, return_full_G2=False):
        """tau and t1 integrals of G2_reuse from the per-t1 rows (reference :484-505)"""
        t1 = self.t1
        t2 = np.linspace(0, self.tend, n_tau + 1)
        g = np.zeros((n_pairs, len(t1)), dtype=complex)
        full = np.zeros((n_pairs, len(t1), n_tau + 1), dtype=complex) if return_full_G2 else None
        # trapezoid over [0, t2[n_t2]] with the row y = (head, tail[0..n_t2)): sum_k d_k (y_k + y_k+1) / 2 as one
        # dot of the tail with the interior weights (the reference's np.trapz per row, without the copies)
        d = np.diff(t2)
        cw = 0.5 * (d[:-1] + d[1:])
        for i, r in enumerate(res):
            n_t2 = n_tau - int(t1[i] / self.dt)
            if return_full_G2:
                rows = self._g2_rows(r, n_pairs, n_t2)
                full[:, i, : n_t2 + 1] = rows
                g[:, i] = _trapz(rows, t2[: n_t2 + 1], axis=1)
                continue
            if n_t2 <= 0:
                continue
            for j in range(n_pairs):
                head = r[1 + n_pairs + j][-(n_t2 + 1)]
                tail = r[1 + j][-n_t2:]
                g[j, i] = 0.5 * d[0] * head + np.dot(tail[:-1], cw[: n_t2 - 1]) + 0.5 * d[n_t2 - 1] * tail[-1]
        if return_full_G2:
            return t1, t2, g, _trapz(g, t1, axis=1), full
        return t1, g, _trapz(g, t1, axis=1)

    @staticmethod
    def _g2_rows(r, n_pairs, n_t2):
        """reference :491-500: tau = 0 from <op1 op2 op3 op4> at t1, tau > 0 from <op2 op3> after t1"""
        rows = np.zeros((n_pairs, n_t2 + 1), dtype=complex)
        for j in range(n_pairs):
            rows[j, 0] = r[1 + n_pairs + j][-(n_t2 + 1)]
            if n_t2 > 0:
                rows[j, 1:] = r[1 + j][-n_t2:]
        return rows

    # ------------------------------------------------------------------ correlation functions
    def G1(self, op1_t, op2_ttau):
        """<op2(t1+tau) op1(t1)> for t1 in self.t1, tau in [0, tend] (reference :162-207)"""
        if op1_t[0] != "(":
            op1_t = "(" + op1_t + ")"
            print("WARNING: added brackets to op1_t")
        if op2_ttau[0] != "(":
            op2_ttau = "(" + op2_ttau + ")"
            print("WARNING: added brackets to op2_ttau")
        t1 = self.t1
        n_tau = int(self.tend / self.dt)
        t2 = np.linspace(0, self.tend, n_tau + 1)
        ends = [t + self.tend for t in t1]
        begins = [max(0, int(round(e / self.dt)) - n_tau) for e in ends]

        def mt(i):
            return [{"operator": op1_t, "applyFrom": "_left", "applyBefore": "false", "time": t1[i]}]
        res = self._batch(lambda i: ends[i], lambda i: begins[i], mt, [op2_ttau, op2_ttau + " * " + op1_t],
                          max(ends) if len(ends) else self.tend)
        G = np.zeros((len(t1), len(t2)), dtype=complex)
        for i, r in enumerate(res):
            G[i, 0] = r[2][-(n_tau + 1)]
            G[i, 1:] = r[1][-n_tau:]
        return t1, t2, G

    def calc_timedynamics(self, output_ops=None):
        opts = dict(self.options)
        if output_ops is not None:
            opts["output_ops"] = output_ops
        return self.system(0, self.tend, **opts)

    def get_spectrum(self, op1_t, op2_ttau, save_g1_dir=None, load=None):
        """spectrum of G1 (reference :215-243): tau-symmetrised FFT for every t1, integrated over t1"""
        if load is not None and os.path.exists(load + "g1.npy"):
            t_axis = np.load(load + "t_axis.npy")
            tau_axis = np.load(load + "tau_axis.npy")
            g1 = np.load(load + "g1.npy")
        else:
            t_axis, tau_axis, g1 = self.G1(op1_t, op2_ttau)
        if save_g1_dir is not None and load is None:
            np.save(save_g1_dir + "g1.npy", g1)
            np.save(save_g1_dir + "t_axis.npy", t_axis)
            np.save(save_g1_dir + "tau_axis.npy", tau_axis)
        dtau = abs(tau_axis[1] - tau_axis[0])
        nt = len(tau_axis)
        freqs = -2 * np.pi * hbar * np.fft.fftfreq(2 * nt - 1, d=dtau)
        sym = np.concatenate([g1[:, ::-1], np.conj(g1[:, 1:])], axis=1)
        spectra = np.fft.fftshift(np.fft.fft(sym, axis=1), axes=1)
        spectrum = np.real(_trapz(spectra.T, t_axis))
        return np.fft.fftshift(freqs), spectrum, spectra

    def G2(self, op1_t, op2_ttau, op3_ttau, op4_t):
        """<op1(t1) op2(t1+tau) op3(t1+tau) op4(t1)> integrated over tau per t1 and then over t1 (reference
        :245-297)"""
        op23 = op2_ttau + " * " + op3_ttau
        n_tau, res = self._g2_runs(op1_t, [op23], op4_t)
        t2 = np.linspace(0, self.tend, n_tau + 1)
        g = np.zeros(len(self.t1), dtype=complex)
        for i, r in enumerate(res):
            n_t2 = n_tau - int(self.t1[i] / self.dt)
            rows = self._g2_rows(r, 1, n_t2)
            g[i] = _trapz(rows[0], t2[: n_t2 + 1])
        return self.t1, g, _trapz(g, self.t1)

    def G2_reuse(self, op1_t, op23s_ttau, op4_t, return_full_G2=False):
        """G2 for several (op2 op3) pairs from one propagation per t1 (reference :423-505)"""
        n_tau, res = self._g2_runs(op1_t, list(op23s_ttau), op4_t)
        return self._reuse_integrals(res, len(op23s_ttau), n_tau, return_full_G2)

    # ------------------------------------------------------------------ two-photon density matrix
    def _pairs_x(self):
        return [self.axdag + " * " + self.ax, self.axdag + " * " + self.ay, self.aydag + " * " + self.ay]

    def _pairs_xy(self):
        return [self.axdag + " * " + self.ax, self.axdag + " * " + self.ay, self.aydag + " * " + self.ax,
                self.aydag + " * " + self.ay]

    @staticmethod
    def _assemble(v, abs_diag=True):
        """4x4 two-photon density matrix (basis xx, xy, yx, yy) from the 10 G2 values, in the index order of
        calc_timedep_data (reference :358-371): 0 xx,xx 1 xx,xy 2 xy,xy 3 xx,yx 4 xx,yy 5 xy,yx 6 xy,yy 7 yx,yx
        8 yx,yy 9 yy,yy; the lower triangle is the conjugate; the diagonal is taken as |.| (:313-333, 385-403)
        except in calc_densitymatrix (:126-156), which keeps the complex values (abs_diag=False)."""
        v = np.asarray(v)
        rho = np.zeros(v.shape[1:] + (4, 4), dtype=complex)
        for (a, b), k in {(0, 0): 0, (3, 3): 9, (1, 1): 2, (2, 2): 7}.items():
            rho[..., a, b] = np.abs(v[k]) if abs_diag else v[k]
        for (a, b), k in {(0, 1): 1, (0, 2): 3, (0, 3): 4, (1, 2): 5, (1, 3): 6, (2, 3): 8}.items():
            rho[..., a, b] = v[k]
            rho[..., b, a] = np.conj(v[k])
        return rho

    def calc_densitymatrix(self):
        """ten separate G2 runs (reference :124-160); returns the concurrence"""
        X, Y, Xd, Yd = self.ax, self.ay, self.axdag, self.aydag
        spec = [(Xd, Xd, X, X), (Xd, Xd, Y, X), (Xd, Yd, Y, X), (Xd, Xd, X, Y), (Xd, Xd, Y, Y),
                (Xd, Yd, X, Y), (Xd, Yd, Y, Y), (Yd, Xd, X, Y), (Yd, Xd, Y, Y), (Yd, Yd, Y, Y)]
        v = [self.G2(*s)[2] for s in spec]
        rho = self._assemble(np.array(v, dtype=complex)[:, None], abs_diag=False)[0]
        return concurrence(rho / np.trace(rho))

    def _reuse_variants(self):
        """the three G2_reuse runs of calc_densitymatrix_reuse: (op1, op23s, op4) = (x, x), (x, y), (y, y)"""
        return [(self.axdag, self._pairs_x(), self.ax), (self.axdag, self._pairs_xy(), self.ay),
                (self.aydag, self._pairs_x(), self.ay)]

    def _densitymatrix_from(self, G, plot_G2=None, return_counts=False, return_rho=False):
        """reference :313-354 from the three G2_reuse results G = [(t1, G_t, G_int)] * 3"""
        (t1, G1t, G1), (t2, G2t, G2), (t3, G3t, G3) = G
        v = np.array([G1[0], G1[1], G1[2], G2[0], G2[1], G2[2], G2[3], G3[0], G3[1], G3[2]])
        rho = self._assemble(v[:, None])[0]
        norm = np.trace(rho)
        if plot_G2 is not None:
            np.save("{}.npy".format(plot_G2), np.array([t1, G1t[0], G1t[1], G1t[2], G2t[0], G2t[1], G2t[2], G2t[3],
                                                        G3t[0], G3t[1], G3t[2]]))
        if return_rho:
            return concurrence(rho / norm), rho
        if return_counts:
            return concurrence(rho / norm), rho[0, 0], rho[1, 1], rho[2, 2], rho[3, 3], rho[0, 3]
        return concurrence(rho / norm)

    def calc_densitymatrix_reuse(self, plot_G2=None, return_counts=False, return_rho=False):
        """three G2_reuse runs (op1, op4) = (x, x), (x, y), (y, y) (reference :299-354)"""
        G = [self.G2_reuse(*v) for v in self._reuse_variants()]
        return self._densitymatrix_from(G, plot_G2, return_counts, return_rho)

    def calc_timedep_data(self):
        """full G2(t, tau) of the 10 components (reference :357-371)"""
        t1, t2, _, _, F1 = self.G2_reuse(self.axdag, self._pairs_x(), self.ax, return_full_G2=True)
        t1, t2, _, _, F2 = self.G2_reuse(self.axdag, self._pairs_xy(), self.ay, return_full_G2=True)
        t1, t2, _, _, F3 = self.G2_reuse(self.aydag, self._pairs_x(), self.ay, return_full_G2=True)
        return t1, t2, np.concatenate([F1, F2, F3], axis=0)

    def calc_timedependent_rho(self, plot_G2=None, t1=None, t2=None, G2_full=None, t=None, G2_t=None, add_norm=0,
                               mode="t", skip=0, return_G2=False):
        """time-resolved two-photon density matrix and concurrence (reference :373-421)"""
        if t is None or G2_t is None:
            if t1 is None or t2 is None or G2_full is None:
                t1, t2, G2_full = self.calc_timedep_data()
            if mode == "t":
                t, G2_t = self.integrate_timedep_G2(t1, t2, G2_full)
            if mode == "tau":
                t, G2_t = self.integrate_g2_tau(t1, t2, G2_full)
        t = t[skip:]
        G2_t = G2_t[:, skip:]
        rho = self._assemble(G2_t)
        rho_int = _trapz(rho, t, axis=0)
        c_int = concurrence(rho_int / np.trace(rho_int).real)
        for k in range(4):
            rho[:, k, k] += add_norm
        norm = np.trace(rho, axis1=1, axis2=2).real
        c_t = np.array([concurrence(rho[i] / norm[i]) for i in range(len(t))], dtype=float)
        if plot_G2 is not None:
            np.savez("{}.npz".format(plot_G2), t1=t1, t2=t2, G2_full=G2_full)
        if return_G2:
            return t, c_t, rho, norm, rho_int, c_int, G2_t
        return t, c_t, rho, norm, rho_int, c_int

    def integrate_g2_tau(self, t1, t2, G2_full):
        """G2(tau) = int dt G2(t, tau) (reference :507-523)"""
        return t2, _trapz(G2_full, t1, axis=1)

    def integrate_timedep_G2(self, t1, t2, G2_full):
        """G2(t) = int_0^t dt' int_0^{t - t'} dtau G2(t', tau) (reference :525-578). The inner integral over the
        tau points with t2 <= t - t' is a prefix of the cumulative trapezoid along tau."""
        t1 = np.asarray(t1)
        t2 = np.asarray(t2)
        dx = np.diff(t2)
        cum = np.zeros_like(G2_full)
        cum[..., 1:] = np.cumsum(0.5 * (G2_full[..., 1:] + G2_full[..., :-1]) * dx, axis=-1)
        G2_t = np.zeros((G2_full.shape[0], len(t1)), dtype=complex)
        for i in range(len(t1)):
            m = np.searchsorted(t2, t1[i] - t1[: i + 1], side="right")     # tau points <= t - t'
            inner = np.where(m > 0, cum[:, np.arange(i + 1), np.maximum(m - 1, 0)], 0.0)
            G2_t[:, i] = _trapz(inner, t1[: i + 1], axis=1)
        return t1, G2_t


_PER_POINT_OPTIONS = {"pulse_file_x", "pulse_file_y", "temp_dir"}


def _same(a, b):
    if a is b:
        return True
    try:
        r = a == b
        return bool(np.all(r)) if isinstance(r, np.ndarray) else bool(r)
    except (ValueError, TypeError):
        try:
            return np.array_equal(np.asarray(a), np.asarray(b))
        except (ValueError, TypeError):
            return False


def _options_differ(a, b):
    """option keys (outside the per-point ones) whose values differ between two instances' options"""
    keys = (set(a) | set(b)) - _PER_POINT_OPTIONS
    return {k for k in keys if (k in a) != (k in b) or not _same(a.get(k), b.get(k))}


def densitymatrix_reuse_scan_sharded(instances, model_kwargs=None, return_rho=False, dist=None, dst=0):
    """`densitymatrix_reuse_scan` over a scan grid sharded across ranks (one process per GPU,
    a contiguous block of grid points per rank, e.g. 32 of 256), gathered to rank `dst` on the device.

    Every rank passes the WHOLE grid (`instances`, `model_kwargs`); rank r runs the points
    scan.shard_range(n, r, world) in its own three launches, packs each point's (concurrence, rho 4 x 4) into 17
    complex values of one device tensor, and scan.gather_tensor sends the blocks to `dst` (RCCL point-to-point over
    xGMI; gloo with host tensors). Returns the full list on `dst` (same order and values as the single-process scan),
    None on the other ranks. The reference runs the same grid as a host loop of per-point ACE runs
    (rabi_rotations.py:172-198 around pol_entanglement/G2.py:301-356)."""
    import torch
    from ..scan import gather_tensor, shard_range
    insts = list(instances)
    kw = list(model_kwargs) if model_kwargs is not None else [{}] * len(insts)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return densitymatrix_reuse_scan(insts, kw, return_rho=return_rho)
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(len(insts), rank, world)
    mine = densitymatrix_reuse_scan(insts[lo:hi], kw[lo:hi], return_rho=True) if hi > lo else []
    packed = np.zeros((len(mine), 17), dtype=np.complex128)
    for i, (c, rho) in enumerate(mine):
        packed[i, 0] = c
        packed[i, 1:] = np.asarray(rho).reshape(16)
    on_dev = dist.get_backend() != "gloo" and torch.cuda.is_available()
    dev = f"cuda:{torch.cuda.current_device()}" if on_dev else "cpu"
    allp = gather_tensor(torch.from_numpy(packed.reshape(-1)).to(dev), dist, dst=dst)
    if rank != dst:
        return None
    allp = allp.cpu().numpy().reshape(-1, 17)
    if len(allp) != len(insts):
        raise RuntimeError(f"gathered {len(allp)} points, expected {len(insts)}")
    out = []
    for row in allp:
        c, rho = float(row[0].real), row[1:].reshape(4, 4)
        out.append((c, rho) if return_rho else c)
    return out


def densitymatrix_reuse_scan(instances, model_kwargs=None, return_rho=False):
    """`calc_densitymatrix_reuse` for every point of a pulse / field scan in three launches in total.

    The reference runs each point on its own (one `PolarizatzionEntanglement` per point, ACE processes per t1 and
    G2_reuse: pol_entanglement/G2.py:299-354, 467-482). Here the instances (one per scan point, each with its own
    pulses / pulse files and t1 grid) share their model callable, dt and tend; `model_kwargs[i]` (e.g. {"bx": 2.0})
    are per-point model keywords the model turns into per-trajectory generators (six_level_system.linear). Each of
    the three G2_reuse variants becomes ONE launch holding every point's t1 trajectories.
    Returns the list of concurrences (with return_rho, (concurrence, rho) pairs), in the order of `instances`."""
    insts = list(instances)
    if not insts:
        return []
    kw = list(model_kwargs) if model_kwargs is not None else [{}] * len(insts)
    if len(kw) != len(insts):
        raise ValueError(f"{len(kw)} model_kwargs for {len(insts)} instances")
    first = insts[0]
    for x in insts[1:]:
        if x.dt != first.dt or x.tend != first.tend:
            raise ValueError("the points of a scan must share dt and tend")
        # every point runs through first.system with first.options: anything else would silently compute a point
        # with another point's model (per-point pulses come from the instance's own pulses / pulse files, per-point
        # model keywords through model_kwargs)
        if x.system is not first.system:
            raise ValueError("the points of a scan must share their model callable (per-point model keywords go in "
                             "model_kwargs)")
        diff = _options_differ(first.options, x.options)
        if diff:
            raise ValueError(f"the points of a scan must share their options; they differ in {sorted(diff)}")
    # the tau integrals on the device (pqd_propagate_trapz: only n_traj x n_pairs values leave it) unless
    # PQD_SCAN_TRAPZ=0 (tables downloaded, integrals on the host as calc_densitymatrix_reuse does)
    on_device = os.environ.get("PQD_SCAN_TRAPZ", "1") != "0"

    def variant(v):
        specs, counts, outs, n_tau = [], [], None, None
        for x, k in zip(insts, kw):
            sp, outs, n_tau = x._g2_specs(*x._reuse_variants()[v])
            for spec in sp:
                spec["pulse_file_x"] = x.options.get("pulse_file_x")
                spec["pulse_file_y"] = x.options.get("pulse_file_y")
                spec.update(k)
            specs += sp
            counts.append(len(sp))
        opts = dict(first.options)
        opts["output_ops"] = outs
        n_pairs = len(first._reuse_variants()[v][1])
        if on_device:
            # G2_reuse's trapezoid over t2 = linspace(0, tend, n_tau + 1) (reference :484-505): head <op1 op2 op3 op4>
            # at t1 (output n_pairs + j), tail <op2 op3> after it (output j); every window is [int(t1/dt), n_tau]
            opts["trapz"] = (list(range(n_pairs, 2 * n_pairs)), list(range(n_pairs)), first.tend / n_tau)
        res = first.system(0, first.tend, trajectories=specs, **opts)
        got, o = [], 0
        for i, x in enumerate(insts):
            if on_device:
                g = np.ascontiguousarray(res[o: o + counts[i]].T)
                got.append((x.t1, g, _trapz(g, x.t1, axis=1)))
            else:
                got.append(x._reuse_integrals(res[o: o + counts[i]], n_pairs, n_tau))
            o += counts[i]
        return got

    # the three launches go through the context lock one at a time; a variant's host work (spec assembly, the
    # tau/t1 integrals) runs beside the next variant's launch
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=3) as ex:
        by_variant = list(ex.map(variant, range(3)))
    per = [[by_variant[v][i] for v in range(3)] for i in range(len(insts))]
    return [x._densitymatrix_from(G, return_rho=return_rho) for x, G in zip(insts, per)]
