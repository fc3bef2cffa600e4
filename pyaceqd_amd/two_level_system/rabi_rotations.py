"""Rabi-rotation scans of the two-level system (pyaceqd/two_level_system/rabi_rotations.py:17-228), on libpqd.

Same class and methods as the reference `RabiRotations`. The reference submits one ACE run per pulse area to a
ThreadPoolExecutor (:172-198); here the whole area scan is ONE launch: every area is a trajectory with its own drive
(`trajectories=[{"pulses": ...}]`, one System per area in a multi-system launch), sharing the PT when phonons are on.
Pulse carving (`carve_pulse`, pyaceqd/pulsegenerator.py lab shaping) and plotting are out of scope:
`carve_pulse=True` raises NotImplementedError, `plot=`/`plot_pulse=` are accepted and ignored; the CSV caches the
reference writes and reads are kept.
"""
import os

import numpy as np

from .. import constants
from ..pulses import ChirpedPulse
from ..tools import export_csv
from .tls import tls

hbar = constants.hbar
temp_dir = constants.temp_dir


def _no_carving(carve_pulse):
    if carve_pulse:
        raise NotImplementedError("carve_pulse needs pyaceqd.pulsegenerator (lab pulse shaping), out of scope "
                                  "(SURVEY.md §2)")


class RabiRotations():
    def __init__(self, dt=0.1, tau=5, area_max=30, n_area=150, gamma_e=1/100, phonons=False, temperature=4, ae=5,
                 ah_ratio=1.15, J_from_file=None, phonon_factor=1, t_mem=10, temp_dir=temp_dir) -> None:
        self.dt = dt
        self.tau = tau
        self.areas = np.linspace(0, area_max, n_area)
        self.gamma_e = gamma_e
        self.phonons = phonons
        self.temperature = temperature
        self.ae = ae
        self.ah_ratio = ah_ratio
        self.J_from_file = J_from_file
        self.phonon_factor = phonon_factor
        self.t_mem = t_mem
        if J_from_file is not None:
            self.pt_name = J_from_file.split(".")[0] + ".ptr"
        else:
            self.pt_name = "pt_T{:.1f}K_AE{:.1f}_AHratio{:.2f}_coupl{:.1f}_dt{:.2f}_tmem{:.1f}.ptr".format(
                self.temperature, self.ae, self.ah_ratio, self.phonon_factor, self.dt, self.t_mem)
        self.full_names = [self.pt_name + s for s in ("_initial", "_initial_0", "_repeated", "_repeated_0", ".npz")]
        self.options = dict({"gamma_e": self.gamma_e, "dt": self.dt, "phonons": self.phonons, "temp_dir": temp_dir,
                             "pt_file": self.pt_name})
        if os.path.exists(self.full_names[0]) or os.path.exists(self.pt_name + ".npz"):
            print("Warning: pt files already exist")

    def _pt_exists(self):
        return os.path.exists(self.pt_name + ".npz") or os.path.exists(self.pt_name + "_initial")

    def delete_pt_files(self):
        for name in self.full_names:
            if os.path.exists(name):
                os.remove(name)

    def get_J_omega(self, plot=False):
        """J(omega) as written by the PT generator's Boson_J_print (reference :43-66)"""
        p = ChirpedPulse(4, 0, t0=20)
        tls(0, 40, p, dt=self.dt, prepare_only=True, phonons=True, ae=self.ae, temperature=self.temperature,
            verbose=False, lindblad=True, temp_dir=self.options["temp_dir"], J_to_file="J_omega.dat",
            factor_ah=self.ah_ratio)
        data = np.loadtxt("J_omega.dat")
        return data[:, 0], data[:, 1]

    def generate_pt(self):
        """generate (and cache under pt_name) the phonon PT for these parameters (reference :68-79)"""
        p1 = ChirpedPulse(tau_0=self.tau, e_start=0, alpha=0, e0=1, polar_x=1.0, t0=4 * self.tau)
        tls(0, 8 * self.tau, p1, dt=self.dt, t_mem=self.t_mem, lindblad=False, phonons=True, factor_ah=self.ah_ratio,
            ae=self.ae, temperature=self.temperature, prepare_only=False, phonon_factor=self.phonon_factor,
            pt_file=self.pt_name, J_file=self.J_from_file)

    def calc_timedynamics(self, tau, area, path="", save=False, plot_pulse=False, detuning=0, tend=None, plot=False,
                          plotlims=None, lindblad=True, carve_pulse=False, pulse_args={"width_t": 4, "central_f": 0},
                          filter_width=0.14):
        """one excitation run (reference :80-112)"""
        _no_carving(carve_pulse)
        p1 = ChirpedPulse(tau_0=tau, e_start=detuning, alpha=0, e0=area, polar_x=1.0, t0=4 * tau)
        if tend is None:
            tend = np.round(10 / self.gamma_e) + 100
        if self.phonons and not self._pt_exists():
            self.generate_pt()
        t, g, x, pgx, pxg = tls(0, tend, p1, lindblad=lindblad, **self.options)
        if save:
            export_csv(path + "timedynamics_{:.2f}ps_{:.2f}pi.csv".format(tau, area), t.real, x.real)
        return t.real, g, x, pgx, pxg

    def _filename(self, path, prefix, carve_pulse, pulse_args, filter_width, carve_fmt):
        name = path + prefix
        if carve_pulse:
            name += carve_fmt.format(pulse_args["width_t"], filter_width)
        if self.phonons:
            name += "{:.1f}K_tau_{:.1f}ps_ae_{:.1f}_ah_{:.2f}_coupl_{:.1f}".format(
                self.temperature, self.tau, self.ae, self.ah_ratio, self.phonon_factor)
        return name

    def _scan(self, system, detuning, integrate, **kw):
        """all areas in one launch: one trajectory (and one System) per pulse area"""
        pulses = [ChirpedPulse(tau_0=self.tau, e_start=detuning, alpha=0, e0=a, polar_x=1.0, t0=4 * self.tau)
                  for a in self.areas]
        tend = np.round(11 / self.gamma_e) if integrate else 8 * self.tau
        specs = [{"pulses": (p,), "t_end": tend} for p in pulses]
        return system(0, tend, lindblad=bool(integrate), trajectories=specs, **kw, **self.options)

    def get_rabi_rotations(self, detuning=0, integrate=True, plot=False, delete_pt=True, path="", workers=15,
                           carve_pulse=False, pulse_args={"width_t": 4, "central_f": 0}, filter_width=0.14,
                           rise_f=0.01, exp_data=None, plot_dynamic=False):
        """emitted photons (gamma_e int x dt) or final x per pulse area (reference :114-228); cached as CSV"""
        _no_carving(carve_pulse)
        filename = self._filename(path, "rabi_", carve_pulse, pulse_args, filter_width, "carve_{:.2f}ps_{:.3f}nm_")
        if os.path.exists(filename + ".csv"):
            data = np.loadtxt(filename + ".csv", delimiter=",")
            return data[:, 0], data[:, 1]
        if self.phonons and not self._pt_exists():
            self.generate_pt()
        runs = self._scan(tls, detuning, integrate)
        results = np.zeros_like(self.areas)
        for i, r in enumerate(runs):
            t, g, x, pgx, pxg = r
            if plot_dynamic:
                d = path + "dynamics/"
                os.makedirs(d, exist_ok=True)
                export_csv(d + "timedynamics_{:.2f}ps_{:.2f}pi.csv".format(self.tau, self.areas[i]), t.real, x.real)
            results[i] = self.gamma_e * np.trapezoid(np.real(x), np.real(t)) if integrate else np.real(x[-1])
        export_csv(filename + ".csv", self.areas, results)
        if delete_pt:
            self.delete_pt_files()
        return self.areas, results
