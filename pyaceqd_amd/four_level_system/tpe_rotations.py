"""Two-photon-excitation (TPE) Rabi scans of the biexciton cascade (pyaceqd/four_level_system/tpe_rotations.py:18-243),
on libpqd.

Same class and methods as the reference `TPERotations`; the area scan the reference fans out over a ThreadPoolExecutor
(:182-207) is one multi-system launch (one trajectory and one System per pulse area). Pulse carving and plotting are
out of scope, as in pyaceqd_amd.two_level_system.rabi_rotations.
"""
import os

import numpy as np

from .. import constants
from ..pulses import ChirpedPulse
from ..tools import export_csv
from ..two_level_system.rabi_rotations import RabiRotations, _no_carving
from .linear import biexciton

hbar = constants.hbar
temp_dir = constants.temp_dir


class TPERotations(RabiRotations):
    def __init__(self, dt=0.1, tau=5, delta_xy=0, delta_b=4, area_max=30, n_area=150, gamma_e=1/100, phonons=False,
                 temperature=4, ae=5, ah_ratio=1.15, J_from_file=None, phonon_factor=1, t_mem=6.1) -> None:
        super().__init__(dt=dt, tau=tau, area_max=area_max, n_area=n_area, gamma_e=gamma_e, phonons=phonons,
                         temperature=temperature, ae=ae, ah_ratio=ah_ratio, J_from_file=J_from_file,
                         phonon_factor=phonon_factor, t_mem=t_mem, temp_dir=temp_dir)
        self.delta_xy = delta_xy
        self.delta_b = delta_b
        self.options.update({"delta_xy": delta_xy, "delta_b": delta_b})

    def get_J_omega(self, plot=False):
        raise NotImplementedError("commented out in the reference (tpe_rotations.py:48-70)")

    def generate_pt(self):
        """biexciton phonon PT for these parameters (reference :72-84)"""
        p1 = ChirpedPulse(tau_0=self.tau, e_start=0, alpha=0, e0=1, polar_x=1.0, t0=4 * self.tau)
        biexciton(0, 8 * self.tau, p1, delta_xy=self.delta_xy, delta_b=self.delta_b, dt=self.dt, t_mem=self.t_mem,
                  lindblad=False, phonons=True, ae=self.ae, temperature=self.temperature, prepare_only=False,
                  pt_file=self.pt_name)

    def calc_timedynamics(self, tau, area, path="", save=False, plot_pulse=False, detuning=0, tend=None, plot=False,
                          plotlims=None, lindblad=True, carve_pulse=False, pulse_args={"width_t": 4, "central_f": 0},
                          filter_width=0.14):
        """one excitation run (reference :86-125): t, |G>, |X>, |Y>, |XX> populations"""
        _no_carving(carve_pulse)
        p1 = ChirpedPulse(tau_0=tau, e_start=detuning, alpha=0, e0=area, polar_x=1.0, t0=4 * tau)
        if tend is None:
            tend = np.round(10 / self.gamma_e) + 100
        if self.phonons and not self._pt_exists():
            self.generate_pt()
        t, g, x, y, b = biexciton(0, tend, p1, lindblad=lindblad, **self.options)
        if save:
            export_csv(path + "timedynamics_{:.2f}ps_{:.2f}pi.csv".format(tau, area), t.real, x.real, y.real, b.real)
        return t.real, g, x, y, b

    def _scan(self, system, detuning, integrate, **kw):
        pulses = [ChirpedPulse(tau_0=self.tau, e_start=detuning, alpha=0, e0=a, polar_x=1.0, t0=4 * self.tau)
                  for a in self.areas]
        tend = np.round(10 / self.gamma_e) + 100 if integrate else 8 * self.tau
        specs = [{"pulses": (p,), "t_end": tend} for p in pulses]
        return system(0, tend, lindblad=bool(integrate), trajectories=specs, **kw, **self.options)

    def get_rabi_rotations(self, detuning=0, integrate=True, plot=False, delete_pt=True, path="", workers=15,
                           carve_pulse=False, pulse_args={"width_t": 4, "central_f": 0}, filter_width=0.14,
                           exp_data=None, plot_dynamic=False):
        """(areas, results[3, n_area]): emitted X, Y, XX photons (XX counted twice) or final populations
        (reference :127-243); cached as CSV"""
        _no_carving(carve_pulse)
        filename = self._filename(path, "tpe_", carve_pulse, pulse_args, filter_width, "carve_{:.1f}ps_{:.1f}nm_")
        if os.path.exists(filename + ".csv"):
            data = np.loadtxt(filename + ".csv", delimiter=",")
            return data[:, 0], data[:, 1], data[:, 2], data[:, 3]
        if self.phonons and not self._pt_exists():
            self.generate_pt()
        runs = self._scan(biexciton, detuning, integrate)
        results = np.zeros([3, len(self.areas)])
        for i, r in enumerate(runs):
            t, g, x, y, b = r
            if plot_dynamic:
                d = path + "dynamics/"
                os.makedirs(d, exist_ok=True)
                export_csv(d + "timedynamics_{:.2f}ps_{:.2f}pi.csv".format(self.tau, self.areas[i]), t.real, x.real)
            if integrate:
                tt = np.real(t)
                results[:, i] = [self.gamma_e * np.trapezoid(np.real(x), tt), self.gamma_e * np.trapezoid(np.real(y), tt),
                                 2 * self.gamma_e * np.trapezoid(np.real(b), tt)]
            else:
                results[:, i] = [x[-1].real, y[-1].real, b[-1].real]
        export_csv(filename + ".csv", self.areas, *results.real)
        if delete_pt:
            self.delete_pt_files()
        return self.areas, results
