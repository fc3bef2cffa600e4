"""Six-level QD G/X/Y/D_x/D_y/B with magnetic fields (pyaceqd/six_level_system/linear.py:20-72), on libpqd.

|0> = G, |1> = X, |2> = Y, |3> = S = D_x, |4> = F = D_y, |5> = B. Same signature, constants and
operator strings as the reference `sixls_linear` (bright-dark coupling from bx, bright-bright /
dark-dark coupling from bz); output_dm=True returns the full density matrix through compose_dm.
"""
import numpy as np

from ..general_system.general_system import system_ace_stream
from ..tools import output_ops_dm, compose_dm
from .. import constants

temp_dir = constants.temp_dir
hbar = constants.hbar
d0 = 0.25  # meV
d1 = 0.12
d2 = 0.05
mu_b = 5.7882818012e-2   # meV/T
g_ex = -0.65  # in plane electron g factor
g_ez = -0.8   # out of plane electron g factor
g_hx = -0.35  # in plane hole g factor
g_hz = -2.2   # out of plane hole g factor

_FWD = ("trajectories", "n_sub", "device", "rho0", "get_M_t", "calc_dynmap", "pulse_sampling", "trapz")


def energies_linear(d0=0.25, d1=0.12, d2=0.05, delta_B=4, delta_E=0.0):
    E_X = delta_E + (d0 + d1) / 2.0
    E_Y = delta_E + (d0 - d1) / 2.0
    E_S = delta_E - (d0 - d2) / 2.0
    E_F = delta_E - (d0 + d2) / 2.0
    E_B = 2. * delta_E - delta_B
    return E_X, E_Y, E_S, E_F, E_B


def sixls_ops(delta_b=4, gamma_e=1/100, gamma_b=None, gamma_d=0, bx=0, bz=0, lindblad=False, rf=False,
              d0=d0, d1=d1, d2=d2):
    """The strings the reference writes for this model (six_level_system/linear.py:41-62)."""
    E_X, E_Y, E_S, E_F, E_B = energies_linear(delta_B=delta_b, d0=d0, d1=d1, d2=d2)
    system_op = ["{}*|1><1|_6 + {}*|2><2|_6 + {}*|3><3|_6 + {}*|4><4|_6 + {}*|5><5|_6".format(E_X, E_Y, E_S, E_F, E_B)]
    if bx != 0:
        system_op.append("{}*(|1><3|_6 + |3><1|_6 )".format(-0.5 * mu_b * bx * (g_ex + g_hx)))
        system_op.append("{}*(|2><4|_6 + |4><2|_6 )".format(-0.5 * mu_b * bx * (g_ex - g_hx)))
    if bz != 0.0:
        system_op.append("-i*{}*(|2><1|_6 - |1><2|_6 )".format(-0.5 * mu_b * bz * (g_ez - 3 * g_hz)))
        system_op.append("-i*{}*(|4><3|_6 - |3><4|_6 )".format(+0.5 * mu_b * bz * (g_ez + 3 * g_hz)))
    boson_op = "1*(|1><1|_6+|2><2|_6+|3><3|_6+|4><4|_6) + 2*|5><5|_6"
    lindblad_ops = []
    if lindblad:
        gb = gamma_e if gamma_b is None else gamma_b
        lindblad_ops = [["|0><1|_6", gamma_e], ["|0><2|_6", gamma_e], ["|1><5|_6", gb], ["|2><5|_6", gb],
                        ["|0><3|_6", gamma_d], ["|0><4|_6", gamma_d]]
    interaction_ops = [["|1><0|_6+|5><1|_6", "x"], ["|2><0|_6+|5><2|_6", "y"]]
    rf_op = "|1><1|_6+|2><2|_6+|3><3|_6+|4><4|_6+2*|5><5|_6" if rf else None
    return system_op, boson_op, lindblad_ops, interaction_ops, rf_op


def sixls_linear(t_start, t_end, *pulses, dt=0.5, delta_b=4, gamma_e=1/100, gamma_b=None, gamma_d=0, bx=0, bz=0,
                 phonons=False, ae=3.0, temperature=4, verbose=False, lindblad=False, temp_dir=temp_dir, pt_file=None,
                 suffix="", multitime_op=None, pulse_file_x=None, pulse_file_y=None, prepare_only=False,
                 output_ops=["|0><0|_6", "|1><1|_6", "|2><2|_6", "|3><3|_6", "|4><4|_6", "|5><5|_6"],
                 initial="|0><0|_6", t_mem=20.48, output_dm=False, dressedstates=False, rf=False, rf_file=None,
                 firstonly=False, calibration_file=None, print_H=False, use_infinite=True, d0=d0, d1=d1, d2=d2,
                 **options):
    if calibration_file is not None:
        raise NotImplementedError("calibration INI files are out of scope (SURVEY.md §2, tools.py:308-346)")
    system_op, boson_op, lindblad_ops, interaction_ops, rf_op = sixls_ops(
        delta_b, gamma_e, gamma_b, gamma_d, bx, bz, lindblad, rf, d0, d1, d2)
    if output_dm:
        output_ops = output_ops_dm(dim=6)
    fwd = {k: options[k] for k in _FWD if k in options}
    if fwd.get("trajectories") is not None:
        # per-trajectory magnetic fields (an e0 x bx scan in one launch): a spec's "bx" / "bz" become its own
        # system_op, the strings this function writes for those fields
        specs, field_ops = [], {}
        for spec in fwd["trajectories"]:
            if "bx" in spec or "bz" in spec:
                spec = dict(spec)
                key = (spec.pop("bx", bx), spec.pop("bz", bz))
                if key not in field_ops:
                    field_ops[key] = sixls_ops(delta_b, gamma_e, gamma_b, gamma_d, key[0], key[1], lindblad, rf,
                                               d0, d1, d2)[0]
                spec["system_op"] = field_ops[key]
            specs.append(spec)
        fwd["trajectories"] = specs
    result = system_ace_stream(
        t_start, t_end, *pulses, dt=dt, phonons=phonons, t_mem=t_mem, ae=ae, temperature=temperature,
        verbose=verbose, temp_dir=temp_dir, pt_file=pt_file, suffix=suffix, multitime_op=multitime_op,
        system_prefix="sixls_linear", threshold="10", threshold_ratio="0.3", buffer_blocksize="-1",
        dict_zero="16", precision="12", boson_e_max=7, system_op=system_op, pulse_file_x=pulse_file_x,
        pulse_file_y=pulse_file_y, boson_op=boson_op, initial=initial, lindblad_ops=lindblad_ops,
        interaction_ops=interaction_ops, output_ops=output_ops, prepare_only=prepare_only,
        dressedstates=dressedstates, rf_op=rf_op, rf_file=rf_file, firstonly=firstonly, print_H=print_H,
        use_infinite=use_infinite, **fwd)
    if output_dm:
        if isinstance(result, list):
            return [compose_dm(r, dim=6) for r in result]
        return compose_dm(result, dim=6)
    return result
