"""Two-level quantum dot (pyaceqd/two_level_system/tls.py:16-77), on libpqd.

Same signature and defaults as the reference `tls`; the operator strings are identical (H on
|1><1|_2 via e_x, x-polarised pulse coupling |1><0|_2, boson operator phonon_factor*|1><1|_2,
radiative decay |0><1|_2, optional pure dephasing). Unknown keywords (`trajectories`, `n_sub`,
`device`) are forwarded to system_ace_stream so the two-time sweeps can batch trajectories.
"""
from ..general_system.general_system import system_ace_stream
from .. import constants

hbar = constants.hbar
temp_dir = constants.temp_dir

_FWD = ("trajectories", "n_sub", "device", "pulse_sampling", "trapz")


def tls(t_start, t_end, *pulses, dt=0.1, gamma_e=1/100, phonons=False, t_mem=6.4, ae=5.0, temperature=4,
        verbose=False, lindblad=False, temp_dir=temp_dir, pt_file=None, suffix="", multitime_op=None,
        pulse_file=None, pulse_file_x=None, prepare_only=False,
        output_ops=["|0><0|_2", "|1><1|_2", "|0><1|_2", "|1><0|_2"], phonon_factor=1.0, LO_params=None,
        dressedstates=False, rf=False, rf_file=None, firstonly=False, dephasing=None, J_to_file=None, J_file=None,
        factor_ah=None, use_infinite=True, threshold=8, calc_dynmap=False, rho0=None, e_x=0, get_M_t=None,
        initial="|0><0|_2", **options):
    system_op = ["({}*|1><1|_2)".format(e_x)] if e_x != 0 else None
    boson_op = "{:.3f}*|1><1|_2".format(phonon_factor)
    lindblad_ops = [["|0><1|_2", gamma_e]] if lindblad else []
    if dephasing is not None:
        lindblad_ops.append(["|0><0|_2-|1><1|_2", dephasing])
    interaction_ops = [["|1><0|_2", "x"]]
    rf_op = "|1><1|_2" if rf else None
    if pulse_file is None and pulse_file_x is not None:
        pulse_file = pulse_file_x
    fwd = {k: options[k] for k in _FWD if k in options}
    return system_ace_stream(
        t_start, t_end, *pulses, dt=dt, phonons=phonons, t_mem=t_mem, ae=ae, temperature=temperature,
        verbose=verbose, temp_dir=temp_dir, pt_file=pt_file, suffix=suffix, multitime_op=multitime_op,
        pulse_file_x=pulse_file, system_prefix="tls", threshold=str(int(threshold)), threshold_ratio="0.3",
        buffer_blocksize="-1", dict_zero="16", precision="12", boson_e_max=7, system_op=system_op,
        boson_op=boson_op, initial=initial, lindblad_ops=lindblad_ops, interaction_ops=interaction_ops,
        output_ops=output_ops, prepare_only=prepare_only, LO_params=LO_params, dressedstates=dressedstates,
        rf_op=rf_op, rf_file=rf_file, firstonly=firstonly, J_to_file=J_to_file, J_file=J_file,
        factor_ah=factor_ah, use_infinite=use_infinite, calc_dynmap=calc_dynmap, rho0=rho0, get_M_t=get_M_t, **fwd)
