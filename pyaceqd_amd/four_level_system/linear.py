"""Four-level biexciton cascade G/X/Y/B (pyaceqd/four_level_system/linear.py:8-39), on libpqd.

|0> = G, |1> = X, |2> = Y, |3> = B. Same signature, defaults and operator strings as the
reference `biexciton`: binding energy delta_b on |3><3|, fine-structure splitting delta_xy,
x/y-polarised ladder couplings, boson operator 1*(|1><1|+|2><2|) + 2*|3><3|, four decay channels.
"""
from ..general_system.general_system import system_ace_stream
from .. import constants

hbar = constants.hbar
temp_dir = constants.temp_dir

_FWD = ("trajectories", "n_sub", "device", "rho0", "get_M_t", "pulse_sampling", "trapz")


def biexciton_ops(delta_xy=0, shift_x=True, coupl_xy=0, delta_b=4, gamma_e=1/100, gamma_b=None, lindblad=False,
                  rf=False):
    """The strings the reference writes for this model (four_level_system/linear.py:13-33)."""
    if shift_x:
        system_op = ["{}*|3><3|_4".format(-delta_b), "{}*|1><1|_4".format(-delta_xy / 2),
                     "{}*|2><2|_4".format(delta_xy / 2)]
    else:
        system_op = ["{}*|3><3|_4".format(-delta_b), "{}*|2><2|_4".format(delta_xy)]
    boson_op = "1*(|1><1|_4 + |2><2|_4) + 2*|3><3|_4"
    lindblad_ops = []
    if lindblad:
        gb = gamma_e if gamma_b is None else gamma_b
        lindblad_ops = [["|0><1|_4", gamma_e], ["|0><2|_4", gamma_e], ["|1><3|_4", gb], ["|2><3|_4", gb]]
    interaction_ops = [["|1><0|_4+|3><1|_4", "x"], ["|2><0|_4+|3><2|_4", "y"]]
    if coupl_xy != 0:
        system_op += ["{}*|1><2|_4".format(coupl_xy), "{}*|2><1|_4".format(coupl_xy)]
    rf_op = "|1><1|_4 + |2><2|_4 + 2*|3><3|_4" if rf else None
    return system_op, boson_op, lindblad_ops, interaction_ops, rf_op


def biexciton(t_start, t_end, *pulses, dt=0.5, delta_xy=0, shift_x=True, coupl_xy=0, delta_b=4, gamma_e=1/100,
              gamma_b=None, phonons=False, ae=3.0, temperature=4, verbose=False, lindblad=False, temp_dir=temp_dir,
              pt_file=None, suffix="", multitime_op=None, pulse_file_x=None, pulse_file_y=None, prepare_only=False,
              output_ops=["|0><0|_4", "|1><1|_4", "|2><2|_4", "|3><3|_4"], initial="|0><0|_4", t_mem=20.48,
              dressedstates=False, rf=False, rf_file=None, firstonly=False, use_infinite=False, calc_dynmap=False,
              **options):
    system_op, boson_op, lindblad_ops, interaction_ops, rf_op = biexciton_ops(
        delta_xy, shift_x, coupl_xy, delta_b, gamma_e, gamma_b, lindblad, rf)
    fwd = {k: options[k] for k in _FWD if k in options}
    return system_ace_stream(
        t_start, t_end, *pulses, dt=dt, phonons=phonons, t_mem=t_mem, ae=ae, temperature=temperature,
        verbose=verbose, temp_dir=temp_dir, pt_file=pt_file, suffix=suffix, multitime_op=multitime_op,
        system_prefix="b_linear", threshold="10", threshold_ratio="0.3", buffer_blocksize="-1", dict_zero="16",
        precision="12", boson_e_max=7, system_op=system_op, pulse_file_x=pulse_file_x, pulse_file_y=pulse_file_y,
        boson_op=boson_op, initial=initial, lindblad_ops=lindblad_ops, interaction_ops=interaction_ops,
        output_ops=output_ops, prepare_only=prepare_only, dressedstates=dressedstates, rf_op=rf_op, rf_file=rf_file,
        firstonly=firstonly, use_infinite=use_infinite, calc_dynmap=calc_dynmap, **fwd)
