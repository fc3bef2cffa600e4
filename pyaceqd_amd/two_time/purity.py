"""Single-photon purity and indistinguishability (pyaceqd/two_time/purity.py:26-822), on libpqd.

Same classes, constructors and methods as the reference (`Purity`, `Indistinguishability`). Differences are in how
the work is issued, not in what is computed:
  * the per-t1 ThreadPoolExecutor fan-outs of G2 / G2_modified / G1 (:115-135, :164-184, :229-247) become one
    batched `system(..., trajectories=[...])` call: every (time-bin repeat, t1) pair is a trajectory of one GPU
    launch, its output window the last n_tau + 1 steps the reference slices out;
  * the dynamical-map paths (`dm=True`) use `calc_dynmap` (N^2 basis trajectories on the GPU), the host time-local
    maps of pyaceqd_amd.tools, and the GPU map-chain sweeps of pyaceqd_amd.two_time.propagate_tau_module
    (calc_onetime_parallel_block, calc_twotime_phonon_block) exactly where the reference calls its Fortran module;
  * the phonon time-local maps for every t1 inside the memory window (`get_dm2_phonons_advanced`, :488-511), which
    the reference runs as parallel ACE processes, run one after the other (each is one GPU launch).
Post-processing (trapezoids, the G0 autocorrelation, purity/indistinguishability ratios) follows :191-198, :260-294,
:776-822.
"""
import numpy as np

from ..pulses import PulseTrain
from ..timebin.timebin import TimeBin
from ..tools import calc_tl_dynmap_pseudo, construct_t, extract_dms, op_to_matrix, simple_t_gaussian
from . import propagate_tau_module
from .. import constants

temp_dir = constants.temp_dir


def _trapz(y, x, axis=-1):
    return np.trapezoid(y, x, axis=axis)


def _g0_autocorr(val, t1, n_t2):
    """G0(tau_j) = int dt val(t) val(t + tau_j) over the t1 window, truncated where val runs out (:273-280)"""
    out = np.zeros(n_t2)
    for j in range(n_t2):
        sh = val[j: j + len(t1)]
        out[j] = _trapz(val[: len(sh)] * sh, t1[: len(sh)])
    return out


class Purity(TimeBin):
    def __init__(self, system, sigma_x, sigma_xdag, *pulses, dt=0.1, tb=800, dt_small=0.1, simple_exp=True,
                 gaussian_t=None, verbose=False, workers=15, t_simul=None, options={}, factor_t=1, factor_tau=2,
                 dt_big=None, add_tend=True) -> None:
        train = PulseTrain(tb, 5, *pulses)
        self.factor_t = factor_t
        self.factor_tau = factor_tau
        super().__init__(system, train, dt=dt, tb=tb, simple_exp=simple_exp, gaussian_t=gaussian_t, verbose=verbose,
                         workers=workers, t_simul=t_simul, options=options)
        self.sigma_x = "(" + sigma_x + ")"
        self.sigma_xdag = "(" + sigma_xdag + ")"
        if "gamma_e" in options:
            self.gamma_e = options["gamma_e"]
        else:
            print("gamma_e not included in options, setting to 100")
            self.options["gamma_e"] = 100
            self.gamma_e = 100
        if dt_big is None:
            dt_big = 10 * dt_small
        if self.gaussian_t is not None:
            self.t1 = simple_t_gaussian(0, self.gaussian_t, self.tb, dt_small, dt_big, *pulses, decimals=1,
                                        exp_part=self.simple_exp, add_tend=add_tend)
        else:
            # the reference passes the pulses positionally after dt_big, so the first one lands in dt_exp (:55)
            self.t1 = construct_t(0, self.tb, dt_small, dt_big, *pulses, simple_exp=self.simple_exp, add_tend=add_tend)
        self.t_axis_complete = np.concatenate([self.t1 + i * self.tb for i in range(factor_t)]) if factor_t \
            else np.array([])
        self.options["pulse_file_x"] = self.pulse_file_x
        self.options["pulse_file_y"] = self.pulse_file_y

    def prepare_pulsefile(self, verbose=False, t_simul=None, plot=False):
        """the pulse train on [0, (factor_t + factor_tau + 1) tb] at dt (reference :69-91)"""
        t_end = (self.factor_t + self.factor_tau + 1) * self.tb if t_simul is None else t_simul
        ts = np.linspace(0, t_end, int(t_end / self.dt) + 1)
        self.pulse_file_x = self.temp_dir + "twotime_pulse_x_{}.dat".format(id(self))
        self.pulse_file_y = self.temp_dir + "twotime_pulse_y_{}.dat".format(id(self))
        px, py = self.pulses[0].get_total_xy(ts)
        self._write(self.pulse_file_x, self.pulse_file_y, ts, np.asarray(px, dtype=complex),
                    np.asarray(py, dtype=complex), verbose)

    def calc_timedynamics(self, output_ops=None, t_end=None):
        opts = dict(self.options)
        if output_ops is not None:
            opts["output_ops"] = output_ops
        if t_end is None:
            t_end = (self.factor_t + self.factor_tau + 1) * self.tb
        return self.system(0, t_end, *self.pulses, **opts)

    # ------------------------------------------------------------------ batched two-time sweeps
    def _sweep(self, mto_templates, output_ops):
        """one trajectory per (time-bin repeat i, t1 point j): MTOs at i tb + t1[j], run to that + factor_tau tb;
        returns (n_tau, list of result arrays) with each window ending at the trajectory's last step"""
        n_tau = self.factor_tau * int(self.tb / self.dt)
        specs, t_ends = [], []
        for i in range(self.factor_t):
            for t in self.t1:
                ta = i * self.tb + t
                te = ta + self.factor_tau * self.tb
                ms = []
                for m in mto_templates:
                    mm = dict(m)
                    mm["time"] = ta
                    ms.append(mm)
                n_end = int(round(te / self.dt))
                specs.append({"multitime_op": ms, "t_end": te, "out_begin": max(0, n_end - n_tau)})
                t_ends.append(te)
        opts = dict(self.options)
        opts["output_ops"] = output_ops
        res = self.system(0, max(t_ends), trajectories=specs, **opts) if specs else []
        return n_tau, res

    def _g2_like(self, out_op1, return_whole):
        left = {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"}
        right = {"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"}
        tau0 = self.sigma_xdag + "*" + out_op1 + "*" + self.sigma_x
        n_tau, res = self._sweep([left, right], [out_op1, tau0])
        t2 = np.linspace(0, self.factor_tau * self.tb, n_tau + 1)
        G = np.zeros((len(res), len(t2)))
        for k, r in enumerate(res):
            G[k, 1:] = np.abs(r[1][-n_tau:])
            G[k, 0] = np.abs(r[2][-(n_tau + 1)])
        if return_whole:
            return self.t1, t2, G
        return t2, _trapz(G, self.t_axis_complete, axis=0)

    def G2(self, return_whole=False, tqdm_options={}):
        """<sigma^dag(t) sigma^dag sigma(t + tau) sigma(t)> integrated over t (reference :101-140)"""
        return self._g2_like(self.sigma_xdag + "*" + self.sigma_x, return_whole)

    def G2_modified(self, out_op1, return_whole=False, tqdm_options={}):
        """G2 with a user-chosen middle operator B (reference :142-189)"""
        return self._g2_like(out_op1, return_whole)

    def calc_purity(self):
        """1 - (area of the tau = 0 peak) / (area of the tau = tb peak) (reference :191-198)"""
        t, g2 = self.G2()
        n_1 = int(0.5 * self.tb / self.dt)
        G21 = 2 * _trapz(g2[:n_1], t[:n_1])
        G22 = _trapz(g2[n_1: 3 * n_1], t[n_1: 3 * n_1])
        return 1 - G21 / G22


class Indistinguishability(Purity):
    def __init__(self, system, sigma_x, sigma_xdag, *pulses, dt=0.1, tb=800, dt_small=0.1, simple_exp=True,
                 gaussian_t=None, verbose=False, workers=15, t_simul=None, options={}, dm=False, sigma_x_mat=None,
                 sigma_xdag_mat=None, t_mem=10, dt_big=None, add_tend=True) -> None:
        self.pulses = pulses
        self.dm = dm
        self.tl_map = None
        self.tl_dms = None
        self.t_mem = t_mem
        self.sigma_x_mat = sigma_x_mat
        self.sigma_xdag_mat = sigma_xdag_mat
        if sigma_x_mat is None or sigma_xdag_mat is None:
            print("WARNING: sigma_x_mat or sigma_xdag_mat not provided, trying to convert sigma_x and sigma_xdag to "
                  "matrices")
            self.sigma_x_mat = op_to_matrix(sigma_x)
            self.sigma_xdag_mat = op_to_matrix(sigma_xdag)
        self.dim = self.sigma_x_mat.shape[0]
        super().__init__(system, sigma_x, sigma_xdag, *pulses, dt=dt, tb=tb, dt_small=dt_small, simple_exp=simple_exp,
                         gaussian_t=gaussian_t, verbose=verbose, workers=workers, t_simul=t_simul, options=options,
                         dt_big=dt_big, add_tend=add_tend)

    # ------------------------------------------------------------------ direct propagation
    def G1(self):
        """|<sigma^dag(t + tau) sigma(t)>|^2 integrated over t (reference :216-258)"""
        left = {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"}
        n_tau, res = self._sweep([left], [self.sigma_xdag, self.sigma_xdag + "*" + self.sigma_x])
        t2 = np.linspace(0, self.factor_tau * self.tb, n_tau + 1)
        G = np.zeros((len(res), len(t2)), dtype=complex)
        for k, r in enumerate(res):
            G[k, 1:] = r[1][-n_tau:]
            G[k, 0] = r[2][-(n_tau + 1)]
        return t2, _trapz(np.abs(G) ** 2, self.t_axis_complete, axis=0)

    def _t_axes(self):
        n_tau = self.factor_tau * int(self.tb / self.dt)
        t2 = np.linspace(0, self.factor_tau * self.tb, n_tau + 1)
        t1 = np.linspace(0, self.factor_t * self.tb, int((self.factor_t * self.tb) / self.dt) + 1)
        return t1, t2

    def simple_propagation(self, return_whole=False):
        """uncorrelated reference G0(tau) from one run of <sigma^dag sigma> (reference :260-294)"""
        tend = (self.factor_t + self.factor_tau) * self.tb
        t1, t2 = self._t_axes()
        opts = dict(self.options)
        opts["output_ops"] = [self.sigma_xdag + "*" + self.sigma_x]
        t, val = self.system(0, tend, suffix=-1, **opts)
        return t2, _g0_autocorr(np.abs(val), t1, len(t2))

    # ------------------------------------------------------------------ time-local dynamical maps
    def _rho0(self):
        rho0 = np.zeros((self.dim, self.dim), dtype=complex)
        rho0[0, 0] = 1
        return rho0

    def _bins(self, first_maps, tl_map, record=False):
        """rho(t) over (factor_t + factor_tau) time bins: in every bin the first maps, then the stationary map
        (reference :311-323, :365-377, :433-446, :456-472)"""
        factors = self.factor_t + self.factor_tau
        len_tb = int(self.tb / self.dt)
        t_total = np.linspace(0, factors * self.tb, factors * len_tb + 1)
        N2 = self.dim ** 2
        rho = np.ones((len(t_total), N2), dtype=complex)
        rho[0] = self._rho0().reshape(N2)
        rho[-1] = self._rho0().reshape(N2)
        used = np.zeros((len(t_total) - 1, N2, N2), dtype=complex) if record else None
        for j in range(factors):
            for i in range(1, len_tb + 1):
                M = first_maps[i - 1] if i < len(first_maps) else tl_map
                rho[i + j * len_tb] = M @ rho[i - 1 + j * len_tb]
                if record:
                    used[i + j * len_tb - 1] = M
        return t_total, rho, used

    def _val(self, rho):
        op = self.sigma_xdag_mat @ self.sigma_x_mat
        return np.real(np.einsum("ij,tji->t", op, rho.reshape(len(rho), self.dim, self.dim)))

    def simple_propagation_tl(self, return_whole=False):
        if self.tl_map is None:
            self.get_tl()
        t1, t2 = self._t_axes()
        _, rho, _ = self._bins(self.tl_dms, self.tl_map)
        return t2, _g0_autocorr(self._val(rho), t1, len(t2))

    def simple_propagation_tl_phonons(self, return_whole=False):
        tl_map, dms = self.get_tl_phonons(mtos=[], t_mtos=[])
        t1, t2 = self._t_axes()
        _, rho, _ = self._bins(dms[0], tl_map)
        return t2, _g0_autocorr(self._val(rho), t1, len(t2))

    def _maps(self, t_end, mtos, memory, t_mtos, suffix=None):
        kw = dict(self.options)
        if suffix is not None:
            kw["suffix"] = suffix
        result, dm = self.system(0, t_end, multitime_op=mtos, calc_dynmap=True, **kw)
        _t = np.round(result[0], 6)
        dm_tl = calc_tl_dynmap_pseudo(dm, _t)
        return extract_dms(dm_tl, _t, memory, t_MTOs=t_mtos)

    def get_tl(self, t_mem=None):
        """time-local maps of one pulse period (reference :395-413)"""
        if t_mem is None:
            t_mem = self.gaussian_t
        if t_mem is None:
            t_mem = self.tb / 2
        memory = self.gaussian_t if self.gaussian_t is not None else self.tb
        tl_map, dms = self._maps(2 * t_mem, [], memory, [])
        self.tl_map = tl_map
        self.tl_dms = dms[0]

    def get_tl_phonons(self, mtos=[], t_mtos=[]):
        """maps over 2.1 (gaussian_t + t_mem) with the MTOs in place (reference :415-424)"""
        tmem = self.gaussian_t + self.t_mem
        tl_map, dms = self._maps(2.1 * tmem, mtos, tmem, t_mtos)
        return tl_map, np.array(dms, dtype=complex)

    def calc_timedynamics_tl_phonons(self):
        tl_map, dms = self.get_tl_phonons(mtos=[], t_mtos=[])
        t_total, rho, _ = self._bins(dms[0], tl_map)
        return t_total, rho.reshape((len(t_total), self.dim, self.dim))

    def calc_timedynamics_tl(self):
        if self.tl_map is None:
            self.get_tl()
        t_total, rho, used = self._bins(self.tl_dms, self.tl_map, record=True)
        self.tl_complete = used
        return t_total, rho.reshape((len(t_total), self.dim, self.dim))

    def _with_time(self, mtos, t):
        out = []
        for m in mtos:
            mm = m.copy()
            mm["time"] = t
            out.append(mm)
        return out

    def get_dm2_phonons(self, mtos, t_mto, suffix=1):
        """maps of the window after an MTO at t_mto (reference :475-486)"""
        _, dms = self._maps(t_mto + self.gaussian_t + self.t_mem + 2 * self.dt, self._with_time(mtos, t_mto),
                            self.gaussian_t + self.t_mem, [t_mto], suffix=suffix)
        return dms[1]

    def get_dm2_phonons_advanced(self, mtos, t_mto, suffix=1):
        """as get_dm2_phonons with a fixed end time and the memory window shrinking with t_mto (reference :488-511)"""
        memory = np.max([self.gaussian_t + self.t_mem - t_mto, self.t_mem])
        _, dms = self._maps(self.gaussian_t + 2 * self.t_mem + 2 * self.dt, self._with_time(mtos, t_mto), memory,
                            [t_mto], suffix=suffix)
        return dms[1]

    def _phonon_block(self, mtos, opA, opB, opC, round_t):
        t_apply = self.gaussian_t + self.t_mem + 5 * self.dt
        tl_map, dms_sep = self.get_tl_phonons(mtos=self._with_time(mtos, t_apply), t_mtos=[t_apply])
        dim = self.sigma_x_mat.shape[0]
        tau_max = self.tb * self.factor_tau
        n_tau = int(tau_max / self.dt)
        tau = np.linspace(0, tau_max, n_tau + 1)
        idx = np.where(self.t1 <= (self.gaussian_t + self.t_mem))[0]
        dms_tauc2 = np.zeros((len(idx), *np.shape(dms_sep[0])), dtype=complex)
        dms_tauc2[:, :] = tl_map
        for i in range(len(idx)):
            t = np.round(self.t1[i], 6) if round_t else self.t1[i]
            part = self.get_dm2_phonons_advanced(mtos, t, i)
            dms_tauc2[i, : np.shape(part)[0]] = part
        _tend = self.t_axis_complete[-1] + tau_max
        t_axis = np.linspace(0, _tend, int(_tend / self.dt) + 1)
        G = propagate_tau_module.calc_twotime_phonon_block(
            dm_taucs2=np.asfortranarray(dms_tauc2.transpose(2, 3, 0, 1)),
            dm_sep1=np.asfortranarray(dms_sep[0].transpose(1, 2, 0)),
            dm_sep2=np.asfortranarray(dms_sep[1].transpose(1, 2, 0)), dm_s=tl_map,
            rho_init=self._rho0().reshape(dim ** 2), n_tb=int(self.tb / self.dt), nx_tau=self.factor_tau, dim=dim,
            opa=opA, opb=opB, opc=opC, time=t_axis, time_sparse=self.t_axis_complete)
        return tau, G

    def G1_tl_phonons(self):
        """G1 from phonon time-local maps + the GPU two-time phonon-block sweep (reference :513-644)"""
        mto = {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"}
        tau, G = self._phonon_block([mto], np.identity(self.sigma_x_mat.shape[0]), self.sigma_xdag_mat,
                                    self.sigma_x_mat, round_t=False)
        return tau, _trapz(np.abs(G) ** 2, self.t_axis_complete, axis=0)

    def G2_tl_phonons(self):
        """G2 from phonon time-local maps + the GPU two-time phonon-block sweep (reference :646-713)"""
        m1 = {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"}
        m2 = {"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"}
        tau, G = self._phonon_block([m1, m2], self.sigma_xdag_mat, self.sigma_xdag_mat @ self.sigma_x_mat,
                                    self.sigma_x_mat, round_t=True)
        return tau, _trapz(np.abs(G), self.t_axis_complete, axis=0)

    def _block_sweep(self, opA, opB, opC):
        if self.tl_map is None:
            self.get_tl()
        dim = self.sigma_x_mat.shape[0]
        tau_max = self.tb * self.factor_tau
        n_tau = int(tau_max / self.dt)
        tau = np.linspace(0, tau_max, n_tau + 1)
        _tend = self.t_axis_complete[-1] + tau_max
        t_axis = np.linspace(0, _tend, int(_tend / self.dt) + 1)
        G = propagate_tau_module.calc_onetime_parallel_block(
            dm_block=np.asfortranarray(self.tl_dms.transpose(1, 2, 0)), dm_s=self.tl_map,
            rho_init=self._rho0().reshape(dim ** 2), n_tb=int(self.tb / self.dt), nx_tau=self.factor_tau, dim=dim,
            opa=opA, opb=opB, opc=opC, time=t_axis, time_sparse=self.t_axis_complete)
        return tau, G

    def G2_tl(self):
        """G2 on the periodic time-local map chain (reference :715-745)"""
        tau, G = self._block_sweep(self.sigma_xdag_mat, self.sigma_xdag_mat @ self.sigma_x_mat, self.sigma_x_mat)
        return tau, _trapz(np.abs(G), self.t_axis_complete, axis=0)

    def G1_tl(self):
        """G1 on the periodic time-local map chain (reference :747-774)"""
        tau, G = self._block_sweep(np.identity(self.sigma_x_mat.shape[0]), self.sigma_xdag_mat, self.sigma_x_mat)
        return tau, _trapz(np.abs(G) ** 2, self.t_axis_complete, axis=0)

    def calc_indistinguishability(self):
        """(indistinguishability, single-photon purity) from the tau = 0 and tau = tb peak areas of G0, G1, G2
        (reference :776-822)"""
        phon = bool(self.options.get("phonons", False)) if self.dm else False
        if self.dm:
            if phon:
                print("Calculating with phonons")
            t, g1 = self.G1_tl_phonons() if phon else self.G1_tl()
        else:
            t, g1 = self.G1()
        n_1 = int(0.5 * self.tb / self.dt)

        def peaks(x, g):
            return 2 * _trapz(g[:n_1], x[:n_1]), _trapz(g[n_1: 3 * n_1], x[n_1: 3 * n_1])
        G11, G12 = peaks(t, g1)
        if self.dm:
            t2, g2 = self.G2_tl_phonons() if phon else self.G2_tl()
        else:
            t2, g2 = self.G2()
        G21, G22 = peaks(t2, g2)
        if self.dm:
            t0, g0 = self.simple_propagation_tl_phonons() if phon else self.simple_propagation_tl()
        else:
            t0, g0 = self.simple_propagation()
        G01, G02 = peaks(t0, g0)
        result = (G01 - G11 + G21) / (G02 - G12 + G22)
        return 1 - result, 1 - G21 / G22
