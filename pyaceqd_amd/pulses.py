"""Laser fields f(t) = envelope(t) * exp(-i phi(t)) with a polarisation split (x, y).

Same classes, constructor arguments and methods as pyaceqd/pulses.py (Pulse :7-86,
AsymmetricPulse :88, ChirpedPulse :105-130, PulseTrain :133-159, CWLaser :161-173,
SmoothRectangle :175). Parity is pinned against the reference's own values on a grid
(tests/golden/pyref_pulses.npz). The samples feed the engine's pulse channels
(general_system.system_ace_stream); the sample grid is finer than the step so that the
exponential-midpoint sub-steps land on sample points.
"""
import numpy as np
from scipy.special import erf

from .constants import hbar as HBAR

_SQRT2PI = np.sqrt(2.0 * np.pi)


class Pulse:
    """Gaussian pulse: e0 exp(-(t-t0)^2 / (2 tau^2)) / (sqrt(2 pi) tau), linear chirp w_gain."""

    def __init__(self, tau, e_start, w_gain=0, t0=0, e0=1, phase=0, polar_x=1, polars=None):
        self.tau = tau
        self.e_start = e_start
        self.w_gain = float(w_gain)
        self.t0 = t0
        self.e0 = e0
        self.phase = phase
        self.freq = None
        self.phase_ = None
        self._set_polarisation(polar_x, polars)

    def _set_polarisation(self, polar_x, polars):
        if polars is None:
            self.polar_x = polar_x
            self.polar_y = np.sqrt(1 - polar_x ** 2)
        else:
            norm = np.hypot(np.abs(polars[0]), np.abs(polars[1]))
            self.polar_x, self.polar_y = polars[0] / norm, polars[1] / norm

    def __repr__(self):
        return "%s(tau=%r, e_start=%r, w_gain=%r, t0=%r, e0=%r)" % (
            type(self).__name__, self.tau, self.e_start, self.w_gain, self.t0, self.e0)

    # -- spectral content
    def get_energy(self):
        return self.e_start, self.w_gain

    def set_energy(self, e_start, w_gain):
        self.e_start, self.w_gain = e_start, w_gain

    def set_frequency(self, f):
        """f(t) -> instantaneous angular frequency (1/ps), overrides the linear chirp"""
        self.freq = f

    def get_frequency(self, t):
        if self.freq is not None:
            return self.freq(t)
        return self.e_start / HBAR + self.w_gain * (t - self.t0)

    def set_phase(self, f):
        self.phase_ = f

    def get_full_phase(self, t):
        if self.phase_ is not None:
            return self.phase_(t)
        dt = t - self.t0
        return (self.e_start / HBAR) * dt + 0.5 * self.w_gain * dt ** 2 + self.phase

    def get_energies(self):
        """energy spread (meV) of the chirp between -tau and +tau"""
        return np.abs(self.get_frequency(self.tau) - self.get_frequency(-self.tau)) * HBAR

    # -- time domain
    def _gauss(self, t, tau):
        return np.exp(-0.5 * ((t - self.t0) / tau) ** 2)

    def get_envelope(self, t):
        return self.e0 * self._gauss(t, self.tau) / (_SQRT2PI * self.tau)

    def get_integral(self, t):
        return 0.5 * self.e0 * (1 - erf((self.t0 - t) / (np.sqrt(2) * self.tau)))

    def get_total(self, t):
        return self.get_envelope(t) * np.exp(-1j * self.get_full_phase(t))

    def copy(self):
        return Pulse(self.tau, self.e_start, self.w_gain, self.t0, self.e0, self.phase, self.polar_x)


class AsymmetricPulse(Pulse):
    """Gaussian rising with tau1 and falling with tau2 (normalised with tau1 on both sides)."""

    def __init__(self, tau1, tau2, e_start, t0=0, e0=1, phase=0, polar_x=1, polars=None):
        self.tau1, self.tau2 = tau1, tau2
        super().__init__(tau1, e_start, w_gain=0, t0=t0, e0=e0, phase=phase, polar_x=polar_x, polars=polars)

    def get_envelope(self, t):
        t = np.asarray(t)
        width = np.where(t <= self.t0, self.tau1, self.tau2)
        return self.e0 * np.exp(-0.5 * ((t - self.t0) / width) ** 2) / (_SQRT2PI * self.tau1)

    def copy(self):
        return AsymmetricPulse(self.tau1, self.tau2, self.e_start, self.t0, self.e0, self.phase, self.polar_x)


class ChirpedPulse(Pulse):
    """Transform-limited width tau_0 stretched by the GDD alpha (ps^2): tau = sqrt(alpha^2/tau_0^2 + tau_0^2),
    chirp rate alpha / (alpha^2 + tau_0^4); area e0 (units of pi, see the -0.5*pi*hbar pulse coupling)."""

    def __init__(self, tau_0, e_start, alpha=0, t0=0, e0=1 * np.pi, polar_x=1, phase=0, polars=None):
        self.tau_0 = tau_0
        self.alpha = alpha
        tau = np.sqrt(alpha ** 2 / tau_0 ** 2 + tau_0 ** 2)
        super().__init__(tau=tau, e_start=e_start, w_gain=alpha / (alpha ** 2 + tau_0 ** 4), t0=t0, e0=e0,
                         polar_x=polar_x, phase=phase, polars=polars)

    def get_parameters(self):
        return "tau: {:.4f} ps , a: {:.4f} ps^-2".format(self.tau, self.w_gain)

    def get_envelope(self, t):
        return self.e0 * self._gauss(t, self.tau) / np.sqrt(2 * np.pi * self.tau * self.tau_0)

    def get_ratio(self):
        return np.sqrt(self.tau / self.tau_0)

    def get_integral(self, t):
        return 0.5 * self.e0 * self.get_ratio() * (1 - erf((self.t0 - t) / (np.sqrt(2) * self.tau)))

    def copy(self):
        return ChirpedPulse(self.tau_0, self.e_start, self.alpha, self.t0, self.e0, self.polar_x, self.phase)


class PulseTrain:
    """n_pulses repetitions (spacing delta_t, offset t_shift) of a group of pulses."""

    def __init__(self, delta_t, n_pulses, *pulses, t_shift=0):
        self.delta_t = delta_t
        self.n_pulses = n_pulses
        self.pulses = list(pulses)
        self.t_shift = t_shift

    def _shifts(self):
        return [self.delta_t * k + self.t_shift for k in range(self.n_pulses)]

    def get_total(self, t):
        field = np.zeros_like(t, dtype=complex)
        for s in self._shifts():
            for p in self.pulses:
                field = field + p.get_total(t - s)
        return field

    def get_total_xy(self, t):
        fx = np.zeros_like(t, dtype=complex)
        fy = np.zeros_like(t, dtype=complex)
        for s in self._shifts():
            for p in self.pulses:
                f = p.get_total(t - s)
                fx = fx + p.polar_x * f
                fy = fy + p.polar_y * f
        return fx, fy


class CWLaser(Pulse):
    """Continuous wave: constant envelope e0, no switch-on."""

    def __init__(self, e0, e_start=0, polar_x=1, phase=0, polars=None):
        super().__init__(tau=5, e_start=e_start, e0=e0, polar_x=polar_x, polars=polars, phase=phase)

    def get_envelope(self, t):
        return self.e0

    def copy(self):
        return CWLaser(self.e0, self.e_start, self.polar_x, self.phase)


class SmoothRectangle(Pulse):
    """Rectangle of length tau centred at t0 with logistic edges of width alpha_onoff."""

    def __init__(self, tau, e_start, w_gain=0, t0=0, e0=1, phase=0, alpha_onoff=0.1, polar_x=1, polars=None):
        self.alpha_onoff = alpha_onoff
        self.alpha = 1 / alpha_onoff
        super().__init__(tau, e_start, w_gain=w_gain, t0=t0, e0=e0, phase=phase, polar_x=polar_x, polars=polars)

    def get_envelope_f(self):
        return self.get_envelope

    def get_envelope(self, t):
        rise = 1 + np.exp(-self.alpha * (t - self.t0 + self.tau / 2))
        fall = 1 + np.exp(-self.alpha * (self.t0 - t + self.tau / 2))
        return self.e0 / (rise * fall)

    def copy(self):
        return SmoothRectangle(self.tau, self.e_start, self.w_gain, self.t0, self.e0, self.phase,
                               self.alpha_onoff, self.polar_x)
