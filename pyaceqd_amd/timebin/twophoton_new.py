"""Time-bin entangled photon pairs from a biexciton cascade (pyaceqd/timebin/twophoton_new.py:18-1148), on libpqd.

Same class, constructor and methods as the reference `TwoPhotonTimebinNew`. What changes is how the work is issued:
  * every correlation the reference computes as one ACE process per t1 point (rho_ee_ee, rho_el_el, rho_el_ll part 1)
    or per (t1, t2 >= t1) pair (four_time, rho_ee_el, rho_el_ll part 2; :409-501, :515-557, :1088-1139) is ONE batched
    launch here: all t1 points, or all n(n+1)/2 pairs, are trajectories of a single GPU sweep whose output windows are
    exactly the values the reference slices (the tail after t1, or only the final step);
  * the time-local-map path (calc_densitymatrix_tl, eell_tl_f, eightops_fortran) calls the GPU four_time /
    four_time_8op kernels of pyaceqd_amd.timebin.timebin_tl with the reference's argument conventions (conjugated,
    Fortran-ordered maps, :114-116, :654-656);
  * propagate_tb_new / four_time_tl (the reference's pure-Python map chain, :737-759, :925-1013) keep their serial
    structure; the binary-power steps go through timebin_tl.utils.fast_propagate on the GPU.
Debug helpers that print and only exist to inspect the Fortran (test_apply_ops :792-820) are not provided.
"""
import numpy as np

from .. import constants
from ..tools import calc_tl_dynmap_pseudo, concurrence, construct_t, op_to_matrix, simple_t_gaussian
from . import timebin_tl
from .timebin import TimeBin

temp_dir = constants.temp_dir

options_example = {"verbose": False, "delta_xd": 4, "gamma_e": 1/65, "lindblad": True, "temp_dir": temp_dir,
                   "phonons": False, "pt_file": "tls_dark_3.0nm_4k_th10_tmem20.48_dt0.02.ptr"}


def _mto(op, side, t):
    return {"operator": op, "applyFrom": side, "applyBefore": "false", "time": t}


class TwoPhotonTimebinNew(TimeBin):
    def __init__(self, system, sigma_x, sigma_xdag, sigma_b, sigma_bdag, *pulses, dt=0.02, dim=5, tb=800,
                 dt_small=0.1, n_tbig=10, dt_exp=None, simple_exp=True, gaussian_t=None, verbose=False, workers=15,
                 simple_t=False, options={}) -> None:
        super().__init__(system, *pulses, dt=dt, tb=tb, simple_exp=simple_exp, gaussian_t=gaussian_t, verbose=verbose,
                         workers=workers, options=options)
        self.gamma_e = options["gamma_e"]
        self.dim = dim
        self.prepare_operators(sigma_x=sigma_x, sigma_xdag=sigma_xdag, sigma_b=sigma_b, sigma_bdag=sigma_bdag,
                               verbose=verbose)
        if self.gaussian_t is not None:
            self.t1 = simple_t_gaussian(0, self.gaussian_t, self.tb, dt_small, n_tbig * dt_small, *self.pulses,
                                        decimals=1, exp_part=self.simple_exp)
        if self.gaussian_t is None or simple_t:
            self.t1 = construct_t(0, self.tb, dt_small, n_tbig * dt_small, dt_exp, *self.pulses,
                                  simple_exp=self.simple_exp)

    def calc_timedynamics(self, output_ops=None):
        opts = self.options.copy()
        if output_ops is not None:
            opts["output_ops"] = output_ops
        return self.system(0, 2 * self.tb, *self.pulses, **opts)

    def prepare_operators(self, sigma_x, sigma_xdag, sigma_b, sigma_bdag, verbose=False):
        self.sigma_x = sigma_x
        self.sigma_xdag = sigma_xdag
        self.x_op = "(" + sigma_xdag + " * " + sigma_x + ")"
        self.sigma_b = sigma_b
        self.sigma_bdag = sigma_bdag
        self.b_op = "(" + sigma_bdag + " * " + sigma_b + ")"
        if verbose:
            print("sigma_x: {}, sigma_xdag: {}, x_op: {}".format(self.sigma_x, self.sigma_xdag, self.x_op))
            print("sigma_b: {}, sigma_bdag: {}, b_op: {}".format(self.sigma_b, self.sigma_bdag, self.b_op))

    # ------------------------------------------------------------------ batched propagation
    def _launch(self, items, output_ops):
        """items: (mtos, t_end, n_keep) per trajectory; the output window holds the last n_keep + 1 steps"""
        specs = []
        for mtos, te, keep in items:
            n_end = int(round(te / self.dt))
            specs.append({"multitime_op": mtos, "t_end": te, "out_begin": max(0, n_end - keep)})
        opts = dict(self.options)
        opts["output_ops"] = output_ops
        return self.system(0, max(te for _, te, _ in items), trajectories=specs, **opts)

    def _g2(self, r, n_t2, use_abs=True):
        """tau = 0 from the second output at t1, tau > 0 from the first output after t1 (:239-247, :1073-1081)"""
        f = np.abs if use_abs else (lambda v: v)
        out = np.zeros(n_t2 + 1, dtype=float if use_abs else complex)
        out[0] = f(r[2][-(n_t2 + 1)])
        if n_t2 > 0:
            out[1:] = f(r[1][-n_t2:])
        return out

    def _pairs(self, mto_fn, t_end_fn, output_ops, j0_second):
        """all (i, j >= i) pairs of the t1 grid in one launch; value = final step of output 1 (output 2 for j = i
        when j0_second); returns G2[i] = int over t2 >= t1 and the (t1, t2) table (:515-557)"""
        t1 = self.t1
        n = len(t1)
        items, idx = [], []
        for i in range(n):
            for j in range(i, n):
                items.append((mto_fn(t1[i], t1[j]), t_end_fn(t1[i], t1[j]), 0))
                idx.append((i, j))
        res = self._launch(items, output_ops)
        table = np.zeros((n, n), dtype=complex)
        for (i, j), r in zip(idx, res):
            table[i, j] = r[2][-1] if (j0_second and j == i) else r[1][-1]
        G = np.array([np.trapezoid(table[i, i:], t1[i:]) for i in range(n)], dtype=complex)
        return G, table

    # ------------------------------------------------------------------ diagonal elements
    def rho_ee_ee(self, add_time=0, use_second_zero=False):
        """<XXdag(t1) Xdag(t2) X(t2) XX(t1)> with t1 <= t2 <= tb, plus the reversed order (:201-278)"""
        t1 = self.t1
        n_tau = int(self.tb / self.dt)
        t2 = np.linspace(0, self.tb, n_tau + 1)
        tend = self.tb + add_time

        def part(output_ops, left_op, right_op):
            items = [([_mto(left_op, "_left", t + add_time), _mto(right_op, "_right", t + add_time)], tend,
                      n_tau - int(t / self.dt)) for t in t1]
            res = self._launch(items, output_ops)
            G = np.zeros(len(t1))
            table = np.zeros((len(t1), len(t2)))
            for i, r in enumerate(res):
                n_t2 = n_tau - int(t1[i] / self.dt)
                v = self._g2(r, n_t2)
                G[i] = np.trapezoid(v, t2[: len(v)])
                table[i, -len(v):] = v
            return G, table
        G1, T1 = part([self.sigma_xdag + "*" + self.sigma_x,
                       self.sigma_bdag + "*" + self.sigma_xdag + "*" + self.sigma_x + "*" + self.sigma_b],
                      self.sigma_b, self.sigma_bdag)
        if use_second_zero:
            return t1, t2, G1, np.trapezoid(G1, t1) * self.gamma_e ** 2, G1, G1 * 0, T1
        G2, T2 = part([self.sigma_bdag + "*" + self.sigma_b, "0*" + self.sigma_xdag], self.sigma_x, self.sigma_xdag)
        G = G1 + G2
        return t1, t2, G, np.trapezoid(G, t1) * self.gamma_e ** 2, G1, G2, T1 + T2

    def rho_ll_ll(self, use_second_zero=False):
        return self.rho_ee_ee(add_time=self.tb, use_second_zero=use_second_zero)

    def rho_el_el(self, output_ops=None, sigma_X=None, sigma_Xdag=None):
        """<XXdag(t1) Xdag(t2 + tb) X(t2 + tb) XX(t1)>, t1 in the early, t2 + tb in the late bin (:286-347)"""
        if output_ops is None:
            output_ops = [self.sigma_xdag + "*" + self.sigma_x,
                          self.sigma_bdag + "*" + self.sigma_xdag + "*" + self.sigma_x + "*" + self.sigma_b]
        if sigma_X is None:
            sigma_X = {"operator": self.sigma_b, "applyFrom": "_left", "applyBefore": "false"}
        if sigma_Xdag is None:
            sigma_Xdag = {"operator": self.sigma_bdag, "applyFrom": "_right", "applyBefore": "false"}
        t1 = self.t1
        n_tau = int(self.tb / self.dt)
        t2 = np.linspace(0, self.tb, n_tau + 1)
        items = []
        for t in t1:
            a, b = dict(sigma_X), dict(sigma_Xdag)
            a["time"] = t
            b["time"] = t
            items.append(([a, b], 2 * self.tb, n_tau))
        res = self._launch(items, output_ops)
        G = np.zeros(len(t1))
        for i, r in enumerate(res):
            v = np.abs(r[1][-n_tau - 1:]).astype(float)
            if i == len(t1) - 1:
                v[0] = np.abs(r[2][-n_tau - 1])
            G[i] = np.trapezoid(v, t2[: len(v)])
        return t1, G, np.trapezoid(G, t1) * self.gamma_e ** 2

    def rho_le_le(self):
        """EL,EL with X <-> XX exchanged (:350-365)"""
        output_ops = [self.sigma_bdag + "*" + self.sigma_b,
                      self.sigma_xdag + "*" + self.sigma_bdag + "*" + self.sigma_b + "*" + self.sigma_x]
        return self.rho_el_el(output_ops=output_ops,
                              sigma_X={"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"},
                              sigma_Xdag={"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"})

    # ------------------------------------------------------------------ coherences
    def four_time(self, output_ops, sigma_1, sigma_2, sigma_3):
        """sigma_1 at t1, sigma_2 at t2 >= t1, sigma_3 at t1 + tb, read out at t2 + tb (:515-557); all pairs in
        one launch. MTOs at equal times act in list order, as ACE applies them in param-file order."""
        def mtos(a, b):
            m1, m2, m3 = dict(sigma_1), dict(sigma_2), dict(sigma_3)
            m1["time"], m2["time"], m3["time"] = a, b, a + self.tb
            return [m1, m2, m3]
        G, table = self._pairs(mtos, lambda a, b: b + self.tb, output_ops, j0_second=True)
        return self.t1, G, np.trapezoid(G, self.t1) * self.gamma_e ** 2, table

    def rho_ee_ll(self, use_second_zero=False):
        """EE,LL coherence, both time orderings (:368-393)"""
        t1, G1, v1, T1 = self.four_time(
            [self.sigma_x, self.sigma_x + "*" + self.sigma_b],
            {"operator": self.sigma_bdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_b, "applyFrom": "_left", "applyBefore": "false"})
        if use_second_zero:
            return t1, G1, v1, G1, G1 * 0, T1
        t1, G2, v2, T2 = self.four_time(
            [self.sigma_bdag, self.sigma_b + "*" + self.sigma_x],
            {"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_bdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"})
        return t1, G1 + G2, v1 + v2, G1, G2, T1 + T2

    def rho_ee_el(self, operators=None):
        """EE,EL coherence (:395-505): part 1 MTOs [b, bdag]@t1, xdag@t2, end t2 + tb; part 2 xdag@t1, [b, bdag]@t2,
        end t1 + tb; the final value of the single output is integrated over t2 >= t1"""
        out = [self.sigma_x]
        b, bdag, xdag = self.sigma_b, self.sigma_bdag, self.sigma_xdag
        if operators is not None:
            if len(operators) != 4:
                raise ValueError("operators must be a list of length 4")
            out = [operators[0]]
            b, bdag, xdag = operators[1], operators[2], operators[3]
        G1, _ = self._pairs(lambda a, c: [_mto(b, "_left", a), _mto(bdag, "_right", a), _mto(xdag, "_right", c)],
                            lambda a, c: c + self.tb, out, j0_second=False)
        G2, _ = self._pairs(lambda a, c: [_mto(xdag, "_right", a), _mto(b, "_left", c), _mto(bdag, "_right", c)],
                            lambda a, c: a + self.tb, out, j0_second=False)
        t1 = self.t1
        return t1, G1 + G2, (np.trapezoid(G1, t1) + np.trapezoid(G2, t1)) * self.gamma_e ** 2, G1, G2

    def rho_ee_le(self):
        return self.rho_ee_el(operators=[self.sigma_b, self.sigma_x, self.sigma_xdag, self.sigma_bdag])

    def rho_el_le(self):
        """EL,LE coherence (:1015-1029)"""
        t1, G1, v1, _ = self.four_time(
            [self.sigma_xdag, self.sigma_xdag + "*" + self.sigma_b],
            {"operator": self.sigma_bdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"},
            {"operator": self.sigma_b, "applyFrom": "_left", "applyBefore": "false"})
        t1, G2, v2, _ = self.four_time(
            [self.sigma_b, self.sigma_xdag + "*" + self.sigma_b],
            {"operator": self.sigma_x, "applyFrom": "_left", "applyBefore": "false"},
            {"operator": self.sigma_bdag, "applyFrom": "_right", "applyBefore": "false"},
            {"operator": self.sigma_xdag, "applyFrom": "_right", "applyBefore": "false"})
        return t1, G1 + G2, v1 + v2, G1, G2

    def rho_el_ll(self, calc_lell=False):
        """EL,LL (or LE,LL with calc_lell) coherence (:1031-1143)"""
        x, xd, b, bd = self.sigma_x, self.sigma_xdag, self.sigma_b, self.sigma_bdag
        t1 = self.t1
        n_tau = int(self.tb / self.dt)
        t2 = np.linspace(0, self.tb, n_tau + 1)
        # part 1 (t1 <= t2): one trajectory per t1
        out1 = [xd + "*" + x, xd + "*" + x + "*" + b]
        r_op, l_op = bd, b
        if calc_lell:
            out1 = [bd + "*" + b, bd + "*" + b + "*" + x]
            r_op, l_op = xd, x
        items = [([_mto(r_op, "_right", t), _mto(l_op, "_left", t + self.tb)], 2 * self.tb,
                  n_tau - int(t / self.dt)) for t in t1]
        res = self._launch(items, out1)
        G1 = np.zeros(len(t1), dtype=complex)
        for i, r in enumerate(res):
            n_t2 = n_tau - int(t1[i] / self.dt)
            v = self._g2(r, n_t2, use_abs=False)
            G1[i] = np.trapezoid(v, t2[: len(v)])
        # part 2 (t2 <= t1): all pairs in one launch
        out2 = [b, xd + "*" + b + "*" + x]
        a_op, l2, r2 = bd, x, xd
        if calc_lell:
            out2 = [x, bd + "*" + x + "*" + b]
            a_op, l2, r2 = xd, b, bd
        G2, _ = self._pairs(lambda a, c: [_mto(a_op, "_right", c), _mto(l2, "_left", a + self.tb),
                                          _mto(r2, "_right", a + self.tb)],
                            lambda a, c: c + self.tb, out2, j0_second=True)
        return t1, G1 + G2, (np.trapezoid(G1, t1) + np.trapezoid(G2, t1)) * self.gamma_e ** 2, G1, G2

    def rho_le_ll(self):
        return self.rho_el_ll(calc_lell=True)

    # ------------------------------------------------------------------ density matrix
    def calc_densitymatrix(self, save_dm=False, save_all=False, filename="densitymatrix", verbose=False,
                           reduced=False, use_second_zero=False):
        """two-photon time-bin density matrix in the basis |ee>, |el>, |le>, |ll> (:38-98)"""
        rho = np.zeros([4, 4], dtype=complex)
        t, _, EEEE, rho[0, 0], EEEE1, EEEE2, _ = self.rho_ee_ee(use_second_zero=use_second_zero)
        _, ELEL, rho[1, 1] = self.rho_el_el()
        _, LELE, rho[2, 2] = self.rho_le_le()
        _, _, LLLL, rho[3, 3], LLLL1, LLLL2, _ = self.rho_ll_ll(use_second_zero=use_second_zero)
        _, EELL, rho[0, 3], EELL1, EELL2, _ = self.rho_ee_ll(use_second_zero=use_second_zero)
        rho[3, 0] = np.conj(rho[0, 3])
        z, z1 = 0 * EEEE, 0 * EEEE1
        EEEL = EELE = ELLE = ELLL = LELL = z
        EEEL1 = EEEL2 = EELE1 = EELE2 = ELLE1 = ELLE2 = ELLL1 = ELLL2 = LELL1 = LELL2 = z1
        if not reduced:
            _, EEEL, rho[0, 1], EEEL1, EEEL2 = self.rho_ee_el()
            _, EELE, rho[0, 2], EELE1, EELE2 = self.rho_ee_le()
            _, ELLE, rho[1, 2], ELLE1, ELLE2 = self.rho_el_le()
            _, ELLL, rho[1, 3], ELLL1, ELLL2 = self.rho_el_ll()
            _, LELL, rho[2, 3], LELL1, LELL2 = self.rho_le_ll()
            for a, b in ((0, 1), (0, 2), (1, 2), (1, 3), (2, 3)):
                rho[b, a] = np.conj(rho[a, b])
        norm = np.trace(rho)
        if save_dm or save_all:
            np.save(filename + "_dm.npy", rho)
        if save_all:
            np.save(filename + "_t.npy", t)
            np.save(filename + "_components.npy",
                    np.stack([EEEE, ELEL, LELE, LLLL, EEEL, EELE, EELL, ELLE, ELLL, LELL], axis=0))
            np.save(filename + "_components_1.npy", np.stack([EEEE1, LLLL1, EEEL1, EELE1, EELL1, ELLE1, ELLL1, LELL1]))
            np.save(filename + "_components_2.npy", np.stack([EEEE2, LLLL2, EEEL2, EELE2, EELL2, ELLE2, ELLL2, LELL2]))
        if verbose:
            fmt = {"complex_kind": lambda v: "%.3f+%.3fj" % (v.real, v.imag)}
            print("density matrix:")
            print(np.array2string(rho, formatter=fmt))
            print("normalized density matrix:")
            print(np.array2string(rho / norm, formatter=fmt))
        return concurrence(rho / norm), rho

    # ------------------------------------------------------------------ time-local dynamical maps
    def _calc_dynmaps(self):
        """per-time-bin dynamical maps E(t, 0) from calc_dynmap runs of gaussian_t + 10 ps, time-localised
        (:559-597)"""
        if self.options.get("phonons", False):
            print("Phonons are enabled in the options. Correlation functions will give wrong results.")
        print("Calculating dynamical maps for time-bins...")
        opts = self.options.copy()
        self.prepare_puslefile_tls()
        opts["pulse_file_x"], opts["pulse_file_y"] = self.pulse_file_x1, self.pulse_file_y1
        result1, dm1 = self.system(0, self.gaussian_t + 10, calc_dynmap=True, **opts)
        opts["pulse_file_x"], opts["pulse_file_y"] = self.pulse_file_x2, self.pulse_file_y2
        result2, dm2 = self.system(0, self.gaussian_t + 10, calc_dynmap=True, **opts)
        print("Dynamical maps calculated.")
        _t1 = np.round(np.real(result1[0]), 6)
        _t2 = np.round(np.real(result2[0]), 6)
        if len(_t1) != len(_t2):
            print("Warning: time axes of dyn. maps are not the same length. Check if anything is wrong.")
        if self.dt < 0.00001:
            print("Warning: very small time-step, time-local map uses truncation of t to 1e-6.")
        dm_tl1 = calc_tl_dynmap_pseudo(dm1, _t1)
        dm_tl2 = calc_tl_dynmap_pseudo(dm2, _t2)
        tl_map = dm_tl1[-1]
        self.precalc_tls = self._calc_binary_steps(tl_map)
        self.dm_tl1 = dm_tl1
        self.dm_tl2 = dm_tl2
        return tl_map, dm_tl1, dm_tl2

    def _calc_binary_steps(self, tl_map):
        """tl_map^(2^k), k = 0..int(log2(tb/dt)) (:599-613)"""
        n_bin = int(np.log2(int(self.tb / self.dt))) + 1
        out = np.zeros([n_bin, tl_map.shape[0], tl_map.shape[1]], dtype=complex)
        out[0] = tl_map
        for i in range(1, n_bin):
            out[i] = out[i - 1] @ out[i - 1]
        return out

    def _fortran_maps(self):
        tl_map, dm_1, dm_2 = self._calc_dynmaps()
        conj_f = lambda a: a.transpose(1, 2, 0).conjugate()  # noqa: E731  (column-major view evolves rho^dag)
        return tl_map, conj_f(dm_1), conj_f(dm_2), conj_f(self._calc_binary_steps(tl_map))

    def calc_densitymatrix_tl(self, save_dm=False, filename="densitymatrix_tl", verbose=False, reduced=True):
        """density matrix from the eight-operator map-chain kernel (:100-181); reduced = diagonal + EE,LL"""
        rho = np.zeros([4, 4], dtype=complex)
        _, dm_1, dm_2, precalc = self._fortran_maps()
        rho0 = self.get_initial_state()
        I = np.eye(rho0.shape[0])
        sx, sxd = op_to_matrix(self.sigma_x), op_to_matrix(self.sigma_xdag)
        sb, sbd = op_to_matrix(self.sigma_b), op_to_matrix(self.sigma_bdag)
        # op_et1l, op_et1r, op_et2l, op_et2r, op_lt1l, op_lt1r, op_lt2l, op_lt2r  (:124-138)
        ops = {"eeee": [sb, sbd, sx, sxd, I, I, I, I], "elel": [sb, sbd, I, I, I, I, sx, sxd],
               "lele": [sx, sxd, I, I, I, I, sb, sbd], "llll": [I, I, I, I, sb, sbd, sx, sxd],
               "eeel": [sb, sbd, I, sxd, I, I, I, sx], "eele": [I, sbd, sx, sxd, I, sb, I, I],
               "elle": [I, sbd, sx, I, sxd, I, I, sb], "elll": [I, sbd, I, I, sb, I, sx, sxd],
               "lell": [I, I, I, sxd, sb, sbd, I, sx], "eell": [I, sbd, I, sxd, sb, I, sx, I]}

        def run(name, **kw):
            return self.eightops_fortran(rho0=rho0, operators=ops[name], precalc_tls=precalc, dm_1=dm_1, dm_2=dm_2,
                                         **kw)[2]
        rho[0, 0] = run("eeee", early_only=True).real
        rho[1, 1] = run("elel").real
        rho[2, 2] = run("lele").real
        rho[3, 3] = run("llll").real
        rho[0, 3] = run("eell")
        rho[3, 0] = rho[0, 3].conjugate()
        if not reduced:
            for (a, b), name, kw in (((0, 1), "eeel", {}), ((0, 2), "eele", {"late_t1_only": True}),
                                     ((1, 2), "elle", {}), ((1, 3), "elll", {}), ((2, 3), "lell", {})):
                rho[a, b] = run(name, **kw)
                rho[b, a] = rho[a, b].conjugate()
        norm = np.trace(rho)
        if save_dm:
            np.save(filename + "_dm.npy", rho)
        return concurrence(rho / norm), rho, rho / norm

    def eightops_fortran(self, rho0, operators, precalc_tls, dm_1, dm_2, early_only=False, late_t1_only=False):
        """G12(t1, t2) from timebin_tl.four_time_8op, integrated over t2 >= t1 and t1 (:706-717)"""
        dim = rho0.shape[0]
        t1 = np.round(self.t1, 6)
        dt = np.round(self.dt, 6)
        G12 = timebin_tl.four_time_8op(dm_1, dm_2, rho0.reshape(dim * dim), t1, precalc_tls, dt, dim, *operators,
                                       early_only, late_t1_only, self.tb)
        G = np.array([np.trapezoid(G12[i, i:], self.t1[i:]) for i in range(len(t1))], dtype=complex)
        return t1, G, np.trapezoid(G, t1) * self.gamma_e ** 2, G12

    def eell_tl_f(self):
        """EE,LL coherence from timebin_tl.four_time (:629-670)"""
        ops = [op_to_matrix(s) for s in (self.sigma_bdag, self.sigma_xdag, self.sigma_b, self.sigma_x)]
        _, dm_1, dm_2, precalc = self._fortran_maps()
        rho_init = self.get_initial_state()
        t1 = np.round(self.t1, 6)
        dim = rho_init.shape[0]
        G12 = timebin_tl.four_time(dm_1, dm_2, rho_init.reshape(dim * dim), t1, precalc, np.round(self.dt, 6), dim,
                                   *ops, self.tb)
        G = np.array([np.trapezoid(G12[i, i:], self.t1[i:]) for i in range(len(t1))], dtype=complex)
        return t1, G, np.trapezoid(G, t1) * self.gamma_e ** 2, G12

    def eell_tl_8ops(self):
        """EE,LL via four_time_8op with early/late operator slots (:672-704). The reference's call passes one logical
        argument too few (:697: `..., False, tb)` lands tb in late_t1_only) and fails; here both flags are False."""
        _, dm_1, dm_2, precalc = self._fortran_maps()
        rho_init = self.get_initial_state()
        dim = rho_init.shape[0]
        I = np.eye(dim)
        ops = [I, op_to_matrix(self.sigma_bdag), I, op_to_matrix(self.sigma_xdag), op_to_matrix(self.sigma_b), I,
               op_to_matrix(self.sigma_x), I]
        return self.eightops_fortran(rho_init, ops, precalc, dm_1, dm_2)

    def get_initial_state(self):
        init = "|0><0|_{dim}".format(dim=self.dim)
        if "initial" in self.options:
            init = self.options["initial"]
            print("Using initial state from options:", init)
        else:
            print("Warning: no initial state given, assuming ground state.")
        return op_to_matrix(init)

    def fast_propagate(self, rho, n):
        """apply tl_map^n through the binary powers (:730-735)"""
        for i, bit in enumerate(reversed(np.binary_repr(n))):
            if bit == "1":
                rho = self.precalc_tls[i] @ rho
        return rho

    def propagate_tb_new(self, t_start, t_stop, rho, dm_tl, verbose=False):
        """explicit maps while they last, then binary powers of the stationary map (:737-759)"""
        t_start = np.round(t_start, 6)
        t_stop = np.round(t_stop, 6)
        n_start = int(np.round(t_start / self.dt))
        n_steps = int(np.round(t_stop / self.dt)) - n_start
        steps_dm = max(0, min(len(dm_tl) - n_start, n_steps))
        if verbose:
            print(f"propagate from {t_start} to {t_stop} using {n_steps} steps of {self.dt}, of which {steps_dm} are "
                  "from dm")
        for _ in range(steps_dm):
            rho = dm_tl[n_start] @ rho
            n_start += 1
            n_steps -= 1
        if n_steps <= 0:       # the Fortran fast_propagate is the identity for n <= 0 (timebin_tl.f90:36)
            return rho
        return timebin_tl.utils.fast_propagate(rho, self.precalc_tls.transpose(1, 2, 0), int(np.round(n_steps)))

    def dynamics_tl(self):
        """rho(t) over both bins on the dt grid (:761-790)"""
        _, dm_tl1, dm_tl2 = self._calc_dynmaps()
        rho0 = self.get_initial_state()
        dim = rho0.shape[0]
        t = np.arange(0, 2 * self.tb, self.dt)
        rho_t = np.zeros([len(t), dim, dim], dtype=complex)
        rho_t[0] = rho0
        n_tb = int(self.tb / self.dt)
        for i in range(len(t) - 1):
            k, dm = (i, dm_tl1) if i < n_tb else (i - n_tb, dm_tl2)
            rho_t[i + 1] = self.propagate_tb_new(k * self.dt, (k + 1) * self.dt, rho_t[i].reshape(dim ** 2),
                                                 dm).reshape(dim, dim)
        return t, rho_t

    def dynamics_tl_t1(self):
        """rho on the t1 grid of both bins via timebin_tl.utils.propagate_tb (:822-843)"""
        _, dm_tl1, dm_tl2 = self._calc_dynmaps()
        rho0 = self.get_initial_state()
        dim = rho0.shape[0]
        n = len(self.t1) - 1
        rho_t = np.zeros([2 * len(self.t1) - 1, dim, dim], dtype=complex)
        rho_t[0] = rho0
        t = [0]
        pre = self.precalc_tls.transpose(1, 2, 0)
        for off, dm, shift in ((0, dm_tl1, 0.0), (n, dm_tl2, self.tb)):
            for i in range(n):
                a, b = np.round(self.t1[i], 6), np.round(self.t1[i + 1], 6)
                rho_t[i + 1 + off] = timebin_tl.utils.propagate_tb(a, b, self.dt, rho_t[i + off].reshape(dim ** 2),
                                                                   dm.transpose(1, 2, 0), pre).reshape(dim, dim)
                t.append(self.t1[i + 1] + shift)
        return np.array(t), rho_t[: len(t)]

    def dynamics_tl_t1_t2(self, t1, t2, sigma_1, sigma_2, sigma_3, take_IDs=False):
        """rho with sigma_1 (right) at t1, sigma_2 (right) at t2 and sigma_3 (left) at t1 + tb on a 1 ps grid; like
        the reference it replaces self.t1 by that grid (:845-888)"""
        m1, m2, m3 = (op_to_matrix(s) for s in (sigma_1, sigma_2, sigma_3))
        if take_IDs:
            d = self.get_initial_state().shape[0]
            m1 = m2 = m3 = np.eye(d, dtype=complex)
        _, dm_tl1, dm_tl2 = self._calc_dynmaps()
        rho0 = self.get_initial_state()
        dim = rho0.shape[0]
        self.t1 = np.round(np.linspace(0, self.tb, int(self.tb / 1) + 1, endpoint=True), 6)
        n = len(self.t1) - 1
        rho_t = np.zeros([2 * len(self.t1) - 1, dim, dim], dtype=complex)
        rho_t[0] = rho0
        t = [0]
        for i in range(n):
            a, b = self.t1[i], self.t1[i + 1]
            r = rho_t[i].copy()
            if a == t1:
                r = r @ m1
            if a == t2:
                r = r @ m2
            rho_t[i + 1] = self.propagate_tb_new(a, b, r.reshape(dim ** 2), dm_tl1).reshape(dim, dim)
            t.append(b)
        for i in range(n):
            a, b = self.t1[i], self.t1[i + 1]
            r = rho_t[i + n].copy()
            if a == t1:
                r = m3 @ r
            rho_t[i + 1 + n] = self.propagate_tb_new(a, b, r.reshape(dim ** 2), dm_tl2).reshape(dim, dim)
            t.append(b + self.tb)
        return np.array(t), rho_t

    def dynamics_tl_t1_t2_f(self, _t1, _t2, sigma_1, sigma_2, sigma_3, take_IDs=False):
        raise NotImplementedError("timebin_tl.dynamics_t1_t2 is a serial debug routine of the reference "
                                  "(timebin_tl.f90:344-397); use dynamics_tl_t1_t2")

    def four_time_tl(self, sigma_1, sigma_2, sigma_3, sigma_4, supply_mats=False):
        """EE,LL-type four-time correlation on the host map chain (:925-1013)"""
        if supply_mats:
            m1, m2, m3, m4 = sigma_1, sigma_2, sigma_3, sigma_4
        else:
            m1, m2, m3, m4 = (op_to_matrix(s) for s in (sigma_1, sigma_2, sigma_3, sigma_4))
        n = len(self.t1)
        table = np.zeros([n, n], dtype=complex)
        print("G2 memory footprint: {} MB".format(table.nbytes / 1024 ** 2))
        _, dm_tl1, dm_tl2 = self._calc_dynmaps()
        self.precalc_tls = self._calc_binary_steps(dm_tl1[-1])
        rho0 = self.get_initial_state()
        dim = rho0.shape[0]
        print("Initial state shape :", rho0.shape)
        self.t1 = np.round(self.t1, 6)
        G = np.zeros(n, dtype=complex)
        P = lambda a, b, r, dm: self.propagate_tb_new(a, b, r.reshape(dim ** 2), dm).reshape(dim, dim)  # noqa: E731
        for i in range(n):
            ta = self.t1[i]
            r = P(0, ta, rho0.copy(), dm_tl1) @ m1
            for j in range(n - i):
                tb2 = self.t1[i + j]
                q = P(ta, tb2, r.copy(), dm_tl1) @ m2
                q = P(tb2, self.tb, q, dm_tl1)
                q = m3 @ P(0, ta, q, dm_tl2)
                q = m4 @ P(ta, tb2, q, dm_tl2)
                table[i, j + i] = np.trace(q)
            G[i] = np.trapezoid(table[i, i:], self.t1[i:])
        return self.t1, G, np.trapezoid(G, self.t1) * self.gamma_e ** 2, table

    def eell_tl(self):
        t1, G, v, T = self.four_time_tl(self.sigma_bdag, self.sigma_xdag, self.sigma_b, self.sigma_x)
        return t1, G, v, G, G * 0, T

    def test_apply_ops(self):
        raise NotImplementedError("debug helper of the reference's Fortran utils (twophoton_new.py:792-820)")
