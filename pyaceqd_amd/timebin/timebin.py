"""Time-bin base class (pyaceqd/timebin/timebin.py:7-99): pulse-file preparation shared by the two-time callers.

The reference writes the summed x/y pulse fields to text files (8 decimals) that every ACE run then reads; the
callers here keep that file protocol because the driver's `pulse_file_x/_y` reading (linear interpolation of the
`%.8f` samples) is part of the reference's numerics (the 1e-8 parity floor). Unlike the
reference's destructor (:89-98), only files this object wrote are removed, never user-supplied ones.
"""
import os

import numpy as np

from .. import constants
from ..tools import export_csv

temp_dir = constants.temp_dir


def _field(pulses, ts):
    px = np.zeros_like(ts, dtype=complex)
    py = np.zeros_like(ts, dtype=complex)
    for p in pulses:
        f = p.get_total(ts)
        px = px + p.polar_x * f
        py = py + p.polar_y * f
    return px, py


class TimeBin():
    def __init__(self, system, *pulses, dt=0.02, tb=800, simple_exp=True, gaussian_t=None, verbose=False, workers=15,
                 t_simul=None, options={}) -> None:
        self._written = []
        self.system = system
        self.dt = dt
        self.options = dict(options)
        self.options["dt"] = dt
        self.tb = tb
        self.simple_exp = simple_exp
        self.gaussian_t = gaussian_t
        self.pulses = pulses
        self.workers = workers      # accepted for signature compatibility; trajectories are batched per launch
        if "temp_dir" in options:
            self.temp_dir = options["temp_dir"]
        else:
            print("temp_dir not included in options, setting to temp_dir specified in constants")
            self.options["temp_dir"] = temp_dir
            self.temp_dir = temp_dir
        o = self.options
        if "pulse_file_x" not in o or "pulse_file_y" not in o or (o["pulse_file_x"] is None
                                                                   and o["pulse_file_y"] is None):
            self.prepare_pulsefile(verbose=verbose, t_simul=t_simul)
            o["pulse_file_x"] = self.pulse_file_x
            o["pulse_file_y"] = self.pulse_file_y
        else:
            self.pulse_file_x = o["pulse_file_x"]
            self.pulse_file_y = o["pulse_file_y"]

    def _write(self, fx, fy, ts, px, py, verbose):
        export_csv(fx, ts, px.real, px.imag, precision=8, delimit=" ", verbose=verbose)
        export_csv(fy, ts, py.real, py.imag, precision=8, delimit=" ", verbose=verbose)
        self._written += [fx, fy]

    def prepare_pulsefile(self, verbose=False, t_simul=None):
        """fields on [0, 2.1 tb) (or [0, t_simul)) at dt/5 (reference :32-47)"""
        t_end = 2.1 * self.tb if t_simul is None else t_simul
        ts = np.arange(0, t_end, step=self.dt / 5)
        self.pulse_file_x = self.temp_dir + "timebin_pulse_x_{}.dat".format(id(self))
        self.pulse_file_y = self.temp_dir + "timebin_pulse_y_{}.dat".format(id(self))
        self._write(self.pulse_file_x, self.pulse_file_y, ts, *_field(self.pulses, ts), verbose)

    def prepare_puslefile_tls(self, verbose=False):
        """per-time-bin pulse files for the time-local map workflow; the second bin is shifted to start at 0
        (reference :49-86; the method name keeps the reference's spelling)"""
        t1 = np.arange(0, self.tb, step=self.dt / 5)
        t2 = np.arange(self.tb, 2 * self.tb, step=self.dt / 5)
        first = [p for p in self.pulses if p.t0 < self.tb]
        second = [p for p in self.pulses if not p.t0 < self.tb]
        self.pulse_file_x1 = self.temp_dir + "timebin_pulse_x_tb1_{}.dat".format(id(self))
        self.pulse_file_y1 = self.temp_dir + "timebin_pulse_y_tb1_{}.dat".format(id(self))
        self.pulse_file_x2 = self.temp_dir + "timebin_pulse_x_tb2_{}.dat".format(id(self))
        self.pulse_file_y2 = self.temp_dir + "timebin_pulse_y_tb2_{}.dat".format(id(self))
        self._write(self.pulse_file_x1, self.pulse_file_y1, t1, *_field(first, t1), verbose)
        self._write(self.pulse_file_x2, self.pulse_file_y2, t2 - self.tb, *_field(second, t2), verbose)

    def __del__(self):
        for f in getattr(self, "_written", []):
            try:
                os.remove(f)
            except OSError:
                pass
