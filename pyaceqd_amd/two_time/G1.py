"""First-order correlations and pulsed Mollow spectra (pyaceqd/two_time/G1.py:15-199), on libpqd.

Same functions and signatures as the reference. `G1_general` fans its t grid out as one trajectory per t point
(the reference: one ACE process per point through a ThreadPoolExecutor, :63-77); here all of them are a single
batched `system(..., trajectories=[...])` launch whose output windows are the last n_tau + 1 steps the reference
slices out (:79-88). `workers` is accepted and ignored. The spectra are the reference's tau-symmetrised FFT integrated
over t (:101-110).
"""
import os

import numpy as np

from .. import constants
from ..tools import construct_t, export_csv
from ..two_level_system.tls import tls

HBAR = constants.hbar
temp_dir = constants.temp_dir


def G1_twols(t0=0, tend=600, tau0=0, tauend=600, dt=0.1, dtau=0.5, *pulses, ae=3.0, temperature=4, gamma_e=1/100,
             phonons=False, pt_file=None, workers=10, temp_dir=temp_dir, coarse_t=False, prepare_only=False,
             simple_exp=False, gaussian_t=False, factor_tau=4, **ops):
    """G1 of the TLS: sigma = |0><1| from the left at t, outputs <|1><1|> (tau = 0) and <|1><0|> (reference :15-34)"""
    ts = np.arange(t0, tend + tauend + dtau, step=dtau)
    print(ts[0], ts[1], ts[-1])
    pulse_file = temp_dir + "tls_G1_pulse.dat"
    f = np.zeros_like(ts, dtype=complex)
    for p in pulses:
        f = f + p.get_total(ts)
    export_csv(pulse_file, ts, f.real, f.imag, precision=8, delimit=" ")
    options = {"gamma_e": gamma_e, "phonons": phonons, "ae": ae, "temperature": temperature, "lindblad": True,
               "pt_file": pt_file, "temp_dir": temp_dir, "pulse_file": pulse_file,
               "output_ops": ["|1><1|_2", "|1><0|_2"]}
    options.update(ops)
    mto = {"operator": "|0><1|_2", "applyFrom": "_left", "applyBefore": "false"}
    return G1_general(t0, tend, tau0, tauend, dt, dtau, *pulses, system=tls, multitime_op=mto, coarse_t=coarse_t,
                      workers=workers, prepare_only=prepare_only, simple_exp=simple_exp, gaussian_t=gaussian_t,
                      factor_tau=factor_tau, **options)


def G1_general(t0=0, tend=600, tau0=0, tauend=600, dt=0.1, dtau=0.02, *pulses, system=tls,
               multitime_op={"operator": "|0><1|_2", "applyFrom": "left"}, coarse_t=False, workers=10,
               prepare_only=False, simple_exp=False, gaussian_t=False, factor_tau=4, **options):
    """G1[i, 0] = <out_1>(t_i) after the MTO, G1[i, k>0] = <out_2>(t_i + k dtau)   (reference :36-89)"""
    t = np.linspace(t0, tend, int((tend - t0) / dt) + 1)
    n_tau = int((tauend - tau0) / dtau)
    tau = np.linspace(tau0, tauend, n_tau + 1)
    if coarse_t:
        # positional as in the reference (:44-48): the first pulse lands in construct_t's dt_exp slot
        if gaussian_t:
            t = construct_t(t0, tend, dt, 3 * dt, *pulses, factor_tau=factor_tau, simple_exp=simple_exp,
                            gaussian_t=True)
        else:
            t = construct_t(t0, tend, dt, 10 * dt, *pulses, simple_exp=simple_exp, gaussian_t=False,
                            factor_tau=factor_tau)
    if options["phonons"]:
        if options["pt_file"] is None or not os.path.exists(options["pt_file"] + "_initial"):
            print("calculating pt file for G1")
            system(0, 40, *pulses, dt=dtau, verbose=True, **options)
        else:
            print("using pt_file {}".format(options["pt_file"]))
        if prepare_only:
            return 0, 0, 0
    specs, ends = [], []
    for ti in t:
        m = dict(multitime_op)
        m["time"] = ti
        te = ti + tauend
        n_end = int(round((te - t0) / dtau))
        specs.append({"multitime_op": [m], "t_end": te, "out_begin": max(0, n_end - n_tau)})
        ends.append(te)
    res = system(t0, max(ends), *pulses, dt=dtau, trajectories=specs, **options)
    G = np.zeros((len(t), len(tau)), dtype=complex)
    for i, r in enumerate(res):
        G[i, 0] = r[1][-n_tau - 1]
        G[i, 1:] = r[2][-n_tau:]
    return t, tau, G


def _t_integrated_spectrum(t_axis, tau_axis, g1):
    """tau-symmetrised FFT per t, integrated over t (reference :101-110)"""
    sym = np.concatenate([g1[:, ::-1], np.conj(g1[:, 1:])], axis=1)
    spectra = np.fft.fftshift(np.fft.fft(sym, axis=1), axes=1)
    return np.real(np.trapezoid(spectra.T, t_axis))


def _save(save_dir, name, freqs, y, z):
    if save_dir is not None:
        np.save(save_dir + "x" + name, freqs)
        np.save(save_dir + "y" + name, y)
        np.save(save_dir + "z" + name, z)


def pulsed_mollow_tls_pulses(pulse, areas, tend=500, tauend=500, dt=0.2, dtau=0.02, gamma_e=1/100, ae=3.0,
                             temperature=4, phonons=False, pt_file="tls_3.0nm_4k_th10_tmem20.48_dt0.02.ptr", workers=7,
                             temp_dir=temp_dir, save_dir=None, prepare_only=False, simple_exp=False, gaussian_t=False,
                             factor_tau=4):
    """pulsed Mollow spectra for a given pulse object over pulse areas (reference :91-117); mutates pulse.e0 as the
    reference does"""
    n_tau = int(tauend / dtau)
    spectra = np.zeros([len(areas), 2 * (n_tau + 1) - 1])
    freqs = np.fft.fftshift(-2 * np.pi * HBAR * np.fft.fftfreq(2 * (n_tau + 1) - 1, d=dtau))
    for i, a in enumerate(areas):
        pulse.e0 = a
        t_axis, tau_axis, g1 = G1_twols(0, tend, 0, tauend, dt, dtau, pulse, ae=ae, gamma_e=gamma_e, coarse_t=True,
                                        phonons=phonons, workers=workers, temperature=temperature, pt_file=pt_file,
                                        temp_dir=temp_dir, prepare_only=prepare_only, simple_exp=simple_exp,
                                        gaussian_t=gaussian_t, factor_tau=factor_tau)
        spectra[i] = _t_integrated_spectrum(t_axis, tau_axis, g1)
        _save(save_dir, "_tau{:.2f}_lifet{:.1f}_det{:.1f}.npy".format(pulse.tau, 1 / gamma_e, pulse.e_start), freqs,
              areas, spectra)
    return freqs, areas, spectra


def pulsed_mollow_tls(pulse_tau, areas, detuning=0, tend=500, tauend=500, dt=0.2, dtau=0.02, gamma_e=1/100, ae=3.0,
                      temperature=4, phonons=False, pt_file="tls_3.0nm_4k_th10_tmem20.48_dt0.02.ptr", workers=7,
                      temp_dir=temp_dir, save_dir=None, prepare_only=False, simple_exp=False, gaussian_t=False,
                      **ops):
    """pulsed Mollow spectra of Gaussian pulses over pulse areas (reference :119-160). As in the reference, the
    coarse_t=True call of G1_twols hands the single pulse to construct_t's dt_exp slot (:44-48), so this raises."""
    from ..pulses import ChirpedPulse
    n_tau = int(tauend / dtau)
    spectra = np.zeros([len(areas), 2 * (n_tau + 1) - 1])
    freqs = np.fft.fftshift(-2 * np.pi * HBAR * np.fft.fftfreq(2 * (n_tau + 1) - 1, d=dtau))
    for i, a in enumerate(areas):
        p1 = ChirpedPulse(tau_0=pulse_tau, e_start=detuning, alpha=0, e0=a, t0=pulse_tau * 4)
        t_axis, tau_axis, g1 = G1_twols(0, tend, 0, tauend, dt, dtau, p1, ae=ae, gamma_e=gamma_e, coarse_t=True,
                                        phonons=phonons, workers=workers, temperature=temperature, pt_file=pt_file,
                                        temp_dir=temp_dir, prepare_only=prepare_only, simple_exp=simple_exp,
                                        gaussian_t=gaussian_t, **ops)
        spectra[i] = _t_integrated_spectrum(t_axis, tau_axis, g1)
        _save(save_dir, "_tau{:.2f}_lifet{:.1f}_det{:.1f}.npy".format(pulse_tau, 1 / gamma_e, detuning), freqs,
              areas, spectra)
    return freqs, areas, spectra


def pulsed_mollow_energy(pulse_tau, detunings, area=3, tend=500, tauend=500, dt=0.2, dtau=0.02, gamma_e=1/100, ae=3.0,
                         temperature=4, phonons=False, pt_file="tls_3.0nm_4k_th10_tmem20.48_dt0.02.ptr", workers=7,
                         temp_dir=temp_dir, save_dir=None, prepare_only=False, simple_exp=False, gaussian_t=False):
    """pulsed Mollow spectra over laser detunings (reference :162-186)"""
    from ..pulses import ChirpedPulse
    n_tau = int(tauend / dtau)
    spectra = np.zeros([len(detunings), 2 * (n_tau + 1) - 1])
    freqs = np.fft.fftshift(-2 * np.pi * HBAR * np.fft.fftfreq(2 * (n_tau + 1) - 1, d=dtau))
    for i, d in enumerate(detunings):
        p1 = ChirpedPulse(tau_0=pulse_tau, e_start=d, alpha=0, e0=area, t0=pulse_tau * 4)
        t_axis, tau_axis, g1 = G1_twols(0, tend, 0, tauend, dt, dtau, p1, ae=ae, gamma_e=gamma_e, coarse_t=True,
                                        phonons=phonons, workers=workers, temperature=temperature, pt_file=pt_file,
                                        temp_dir=temp_dir, prepare_only=prepare_only, simple_exp=simple_exp,
                                        gaussian_t=gaussian_t)
        spectra[i] = _t_integrated_spectrum(t_axis, tau_axis, g1)
        _save(save_dir, "_tau{:.2f}_lifet{:.1f}_area{:.1f}.npy".format(pulse_tau, 1 / gamma_e, area), freqs,
              detunings, spectra)
    return freqs, detunings, spectra


def simple_vhom(tend=600, tauend=600, dt=0.1, dtau=0.02, *pulses, ae=3.0, temperature=4, gamma_e=1/100, phonons=False,
                pt_file=None, workers=10, temp_dir=temp_dir, coarse_t=False, prepare_only=False):
    """HOM visibility estimate 2 int |G1|^2 / brightness (reference :188-199, marked 'not tested' there)"""
    options = {"gamma_e": gamma_e, "phonons": phonons, "ae": ae, "temperature": temperature, "lindblad": True,
               "pt_file": pt_file, "temp_dir": temp_dir, "stream": True, "output_ops": ["|1><1|_2"]}
    t, x = tls(0, tend, *pulses, dt=dtau, **options)
    brightness = np.trapezoid(x, t)
    t, tau, g1 = G1_twols(0, tend, 0, tauend, dt, dtau, *pulses, ae=ae, temperature=temperature, gamma_e=gamma_e,
                          phonons=phonons, pt_file=pt_file, workers=workers, temp_dir=temp_dir, coarse_t=coarse_t,
                          prepare_only=prepare_only)
    g1_tau = np.trapezoid(np.abs(g1) ** 2, t)
    return 2 * np.trapezoid(g1_tau, tau) / brightness
