"""The C-ABI library loads on a CPU-only host and exports every entry point include/pqd.h declares
(no compute calls here: those need the GPU)."""
import ctypes as C
import os
import re

import pytest

from pyaceqd_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "pqd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pqd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("pqd_propagate", "pqd_plan_create", "pqd_calc_onetime_parallel", "pqd_four_time_8op",
                 "pqd_pt_create", "pqd_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libpqd.so not built (run __graft_entry__.build())")
    L = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared()) == set(_lib.EXPORTED)


def test_no_device_errors_cleanly():
    """without a GPU the product fails loudly (no CPU fallback)"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises((ValueError, _lib.PQDError)):
        _lib.Context(0)
    assert _lib.lib().pqd_version() >= 1
    assert isinstance(_lib.lib().pqd_last_error(), bytes)
