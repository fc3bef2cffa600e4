"""ctypes binding of libpqd.so (C-ABI declared in include/pqd.h).

The library is built in-tree (pyaceqd_amd/libpqd.so, see __graft_entry__.build()). There is no CPU
fallback: if the library or a gfx950 device is missing, every call raises.
"""
import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PQD_LIB") or os.path.join(_HERE, "libpqd.so")  # PQD_LIB: A/B of builds


class PQDError(RuntimeError):
    code = None  # the PQD_ERR_* status that raised it


PQD_ERR_UNSUPPORTED = 3


class NumericError(PQDError):
    """PQD_ERR_NUMERIC: a propagated output value is NaN or Inf"""


class c128(C.Structure):
    _fields_ = [("re", C.c_double), ("im", C.c_double)]


P_C128 = C.POINTER(c128)
P_I32 = C.POINTER(C.c_int32)
P_I64 = C.POINTER(C.c_int64)
P_F64 = C.POINTER(C.c_double)


class pqd_system(C.Structure):
    _fields_ = [("dim", C.c_int32), ("hbar", C.c_double), ("H0", P_C128),
                ("n_lind", C.c_int32), ("lind_rates", P_F64), ("lind_ops", P_C128),
                ("n_chan", C.c_int32), ("chan_ops", P_C128), ("chan_samples", P_C128),
                ("n_samples", C.c_int32), ("sample_t0", C.c_double), ("sample_dt", C.c_double)]


class pqd_grid(C.Structure):
    _fields_ = [("ta", C.c_double), ("dt", C.c_double), ("n_steps", C.c_int32), ("n_sub", C.c_int32)]


class pqd_pt_desc(C.Structure):
    _fields_ = [("chi", C.c_int32), ("D", C.c_int32), ("n_slices", C.c_int32), ("Q", P_C128),
                ("closure", P_C128), ("closure0", P_C128), ("bond0", P_C128), ("gmap", P_I32)]


class pqd_ace_pt_dims(C.Structure):
    _fields_ = [("n_init", C.c_int32), ("n_slices", C.c_int32), ("chi", C.c_int32), ("D", C.c_int32)]


class pqd_traj(C.Structure):
    _fields_ = [("n_traj", C.c_int32), ("out_begin", P_I32), ("out_end", P_I32), ("out_offset", P_I64),
                ("n_mto", C.c_int32), ("mto_traj", P_I32), ("mto_step", P_I32), ("mto_before", P_I32),
                ("mto_kind", P_I32), ("mto_ops", P_C128)]


_lib = None
_lock = threading.RLock()

_SIGS = {
    "pqd_version": ([], C.c_int32),
    "pqd_last_error": ([], C.c_char_p),
    "pqd_hip_versions": ([P_I32, P_I32], C.c_int),
    "pqd_ctx_create": ([C.c_int32, C.POINTER(C.c_void_p)], C.c_int),
    "pqd_ctx_destroy": ([C.c_void_p], None),
    "pqd_ctx_synchronize": ([C.c_void_p], C.c_int),
    "pqd_pt_create": ([C.c_void_p, C.c_int32, C.POINTER(pqd_pt_desc), C.POINTER(C.c_void_p)], C.c_int),
    "pqd_pt_destroy": ([C.c_void_p], None),
    "pqd_ace_pt_shape": ([C.c_char_p, C.c_int32, C.POINTER(pqd_ace_pt_dims)], C.c_int),
    "pqd_ace_pt_read": ([C.c_char_p, C.c_int32, C.POINTER(pqd_ace_pt_dims), P_C128, P_C128, P_C128, P_C128, P_I32],
                        C.c_int),
    "pqd_free_propagators": ([C.c_void_p, C.POINTER(pqd_system), C.POINTER(pqd_grid), P_C128], C.c_int),
    "pqd_propagate": ([C.c_void_p, C.POINTER(pqd_system), C.POINTER(pqd_grid), C.c_void_p, P_I32, P_C128,
                       C.c_int32, P_C128, C.POINTER(pqd_traj), P_C128, C.c_int64], C.c_int),
    "pqd_propagate_multi": ([C.c_void_p, C.c_int32, C.POINTER(pqd_system), P_I32, C.POINTER(pqd_grid), C.c_void_p,
                             P_I32, P_C128, C.c_int32, P_C128, C.POINTER(pqd_traj), P_C128, C.c_int64], C.c_int),
    "pqd_propagate_table": ([C.c_void_p, C.c_int32, C.POINTER(pqd_system), P_I32, C.POINTER(pqd_grid), C.c_void_p,
                             P_I32, P_C128, C.c_int32, P_C128, C.POINTER(pqd_traj), P_C128, C.c_int64], C.c_int),
    "pqd_propagate_trapz": ([C.c_void_p, C.c_int32, C.POINTER(pqd_system), P_I32, C.POINTER(pqd_grid), C.c_void_p,
                             P_I32, P_C128, C.c_int32, P_C128, C.POINTER(pqd_traj), C.c_int32, P_I32, P_I32,
                             C.c_double, P_C128], C.c_int),
    "pqd_plan_create_multi": ([C.c_void_p, C.c_int32, C.POINTER(pqd_system), P_I32, C.POINTER(pqd_grid),
                               C.c_void_p, P_I32, P_C128, C.c_int32, P_C128, C.POINTER(pqd_traj), C.c_int64,
                               C.POINTER(C.c_void_p)], C.c_int),
    "pqd_plan_create": ([C.c_void_p, C.POINTER(pqd_system), C.POINTER(pqd_grid), C.c_void_p, P_I32, P_C128,
                         C.c_int32, P_C128, C.POINTER(pqd_traj), C.c_int64, C.POINTER(C.c_void_p)], C.c_int),
    "pqd_plan_execute": ([C.c_void_p, C.c_int32], C.c_int),
    "pqd_plan_output_device": ([C.c_void_p], C.c_void_p),
    "pqd_plan_synchronize": ([C.c_void_p], C.c_int),
    "pqd_plan_download": ([C.c_void_p, P_C128, C.c_int64], C.c_int),
    "pqd_plan_copy_output": ([C.c_void_p, C.c_void_p, C.c_int64], C.c_int),
    "pqd_plan_table_len": ([C.c_void_p, P_I64], C.c_int),
    "pqd_plan_download_table": ([C.c_void_p, P_C128, C.c_int64], C.c_int),
    "pqd_plan_trapz": ([C.c_void_p, C.c_int32, P_I32, P_I32, C.c_double, P_C128], C.c_int),
    "pqd_plan_windows": ([C.c_void_p, P_I32], C.c_int),
    "pqd_plan_info": ([C.c_void_p, P_I32, P_I32, P_I32, P_I64], C.c_int),
    "pqd_plan_timing": ([C.c_void_p, P_F64, P_F64, P_I32, C.c_int32], C.c_int),
    "pqd_plan_destroy": ([C.c_void_p], None),
    "pqd_propagate_tau": ([C.c_void_p, P_C128, C.c_int32, P_C128, C.c_int32, C.c_int32, C.c_int32, P_C128], C.c_int),
    "pqd_calc_onetime_parallel": ([C.c_void_p, P_C128, P_C128, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                   P_C128, P_C128, P_C128, P_F64, P_F64, P_C128], C.c_int),
    "pqd_calc_onetime_parallel_block": ([C.c_void_p, P_C128, P_C128, P_C128, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_int32, C.c_int32, P_C128, P_C128, P_C128, P_F64, P_F64,
                                         P_C128], C.c_int),
    "pqd_calc_twotime_phonon_block": ([C.c_void_p, P_C128, P_C128, P_C128, P_C128, P_C128, C.c_int32, C.c_int32,
                                       C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P_C128, P_C128,
                                       P_C128, P_F64, P_F64, P_C128], C.c_int),
    "pqd_four_time_8op": ([C.c_void_p, P_C128, P_C128, P_C128, P_F64, P_C128, C.c_int32, C.c_double, C.c_int32,
                           C.c_int32, P_C128, C.c_int32, C.c_int32, C.c_double, C.c_int32, P_C128], C.c_int),
    "pqd_four_time_8op_rows": ([C.c_void_p, P_C128, P_C128, P_C128, P_F64, P_C128, C.c_int32, C.c_double,
                                C.c_int32, C.c_int32, P_C128, C.c_int32, C.c_int32, C.c_double, C.c_int32, C.c_int32,
                                C.c_int32, P_C128], C.c_int),
    "pqd_four_time": ([C.c_void_p, P_C128, P_C128, P_C128, P_F64, P_C128, C.c_int32, C.c_double, C.c_int32,
                       C.c_int32, P_C128, C.c_double, C.c_int32, P_C128], C.c_int),
    "pqd_dynamics_t1": ([C.c_void_p, P_C128, P_C128, P_C128, P_F64, P_C128, C.c_int32, C.c_double, C.c_int32,
                         C.c_int32, C.c_double, C.c_int32, P_C128], C.c_int),
    "pqd_tl_dynmap_pseudo": ([C.c_void_p, P_C128, C.c_int32, C.c_int32, C.c_double, P_C128], C.c_int),
    "pqd_map_tail": ([C.c_void_p, P_C128, C.c_int32, P_C128, C.c_int32, P_C128, C.c_int32, P_C128], C.c_int),
    # PT generator factorizations on device pointers (ptgen_gpu.py)
    "pqd_ptg_qr": ([C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                    C.c_void_p, P_I32], C.c_int),
    "pqd_ptg_jacobi": ([C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                        C.c_int32, P_I32], C.c_int),
    "pqd_ptg_counters": ([P_I32], C.c_int),
    "pqd_ptg_qr_counters": ([P_I32], C.c_int),
}

EXPORTED = tuple(_SIGS)


def _torch_runtime_first():
    """One HIP runtime per process: torch's ROCm wheel bundles its own libamdhip64 under the soname libpqd links, and
    whichever library loads first serves both. If libpqd came first, torch.cuda.is_available() turned False later in
    the process (the GPU PT generator and the sharded scans use torch device tensors; seen when a process ran libpqd
    propagations before its first generator call). Importing torch (no device initialisation) before libpqd makes
    the order the working one in every process. PQD_TORCH_FIRST=0 skips it; without torch nothing changes."""
    if os.environ.get("PQD_TORCH_FIRST", "1") == "0":
        return
    try:
        import torch  # noqa: F401
    except Exception:  # torch absent or broken: libpqd runs on its own runtime
        pass


def lib():
    """Load libpqd.so (raises PQDError if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise PQDError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
                _torch_runtime_first()
                L = C.CDLL(LIB_PATH)
                for name, (args, res) in _SIGS.items():
                    if os.environ.get("PQD_LIB") and not hasattr(L, name):
                        continue  # A/B against an older build: entry points it predates stay unbound
                    f = getattr(L, name)
                    f.argtypes = args
                    f.restype = res
                _lib = L
                _check_runtime(L)
    return _lib


RUNTIME_VERSIONS = None  # (HIP version libpqd was built against, the loaded runtime's), HIP_VERSION encoding


def _check_runtime(L):
    """with torch imported first, libpqd binds to torch's bundled HIP runtime. The versions are kept in
    RUNTIME_VERSIONS; a different MAJOR version warns (this image pairs ROCm 7.2 with torch's 7.0 runtime, a minor
    difference every GPU test and bench run has used; HIP_VERSION = major 1e7 + minor 1e5 + patch)"""
    global RUNTIME_VERSIONS
    if not hasattr(L, "pqd_hip_versions"):
        return
    b, r = C.c_int32(), C.c_int32()
    if L.pqd_hip_versions(C.byref(b), C.byref(r)) != 0:
        return
    RUNTIME_VERSIONS = (b.value, r.value)
    if b.value // 10000000 != r.value // 10000000:
        import warnings
        warnings.warn(f"libpqd was built against HIP {b.value // 10000000}.{b.value // 100000 % 100} but the process "
                      f"runs HIP runtime {r.value // 10000000}.{r.value // 100000 % 100} (loaded first, e.g. by torch); "
                      f"PQD_TORCH_FIRST=0 keeps libpqd's own runtime", RuntimeWarning, stacklevel=3)


def check(rc):
    if rc != 0:
        msg = lib().pqd_last_error().decode(errors="replace")
        exc = ValueError if rc == 1 else NumericError if rc == 5 else PQDError
        e = exc(f"libpqd error {rc}: {msg}")
        e.code = rc  # the C-ABI status (include/pqd.h PQD_ERR_*)
        raise e


def cptr(a):
    """pointer to a C-contiguous complex128 array (None -> NULL)"""
    if a is None:
        return None
    assert a.dtype == np.complex128 and a.flags["C_CONTIGUOUS"], "need C-contiguous complex128"
    return a.ctypes.data_as(P_C128)


def fptr(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(P_F64)


def iptr(a):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(P_I32)


def lptr(a):
    assert a.dtype == np.int64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(P_I64)


class Context:
    """One HIP device + stream. Calls are serialised per context (the reference's thread-pool callers
    may call in from many threads)."""

    def __init__(self, device=0):
        self.device = int(device)
        h = C.c_void_p()
        check(lib().pqd_ctx_create(self.device, C.byref(h)))
        self.handle = h
        self.lock = threading.RLock()

    def synchronize(self):
        check(lib().pqd_ctx_synchronize(self.handle))

    def __del__(self):
        try:
            if getattr(self, "handle", None) and _lib is not None:
                _lib.pqd_ctx_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


_contexts = {}


def context(device=None):
    """Process-wide default context for `device` (LOCAL_RANK or 0 by default)."""
    if device is None:
        device = int(os.environ.get("PQD_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    with _lock:
        if device not in _contexts:
            try:
                _contexts[device] = Context(device)
            except ValueError:
                # fewer visible devices than LOCAL_RANK (one device exported per rank): use device 0
                if device == 0:
                    raise
                _contexts[device] = _contexts[0] if 0 in _contexts else Context(0)
        return _contexts[device]
