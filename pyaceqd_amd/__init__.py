"""pyaceqd_amd — MI355X-native process-tensor propagator behind pyaceqd's driver API.

The package mirrors the parts of pyaceqd that sit on the propagation hot path
(general_system.system_ace_stream, the 2/4/6-level model wrappers, two_time correlation sweeps,
the f2py sweep modules) and lowers them onto libpqd.so (HIP kernels for gfx950).
"""
from . import constants  # noqa: F401

__version__ = "0.1.0"
