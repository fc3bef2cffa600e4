"""ACE's own process-tensor files: `<name>_initial`, `<name>_initial_0`, `<name>_repeated`, `<name>_repeated_0`.

The reference writes them with ACE (`dont_propagate true` + `write_PT <name>`, general_system.py:152-197), detects
them by `<name>_initial` (:153-156) and hands `add_PT <name>` to the propagation (:236). ACE's binary layout is not
documented anywhere the reference or this container holds, and no ACE-made file exists here (SURVEY.md §8c, §8f
rank 2). libpqd therefore reads ONE stated layout assumption, "ACE_PTB_V0" (pqd_ace_pt_shape / pqd_ace_pt_read,
include/pqd.h; layout in pyaceqd_amd/csrc/ace_pt.cpp and INTEGRATION.md), and refuses anything else with
PQD_ERR_UNSUPPORTED naming the file and the mismatch. `write_ace_pt` writes the same layout (export, round trips).
This is NOT a parity claim: the day an ACE-made file is at hand, the reader's assumption is what to check first.
"""
import os
import struct

import numpy as np

from . import _lib
from .engine import ProcessTensor


def ace_pt_exists(name):
    """the reference's detection (general_system.py:153, 156)"""
    return os.path.exists(str(name) + "_initial")


def read_ace_pt(name, dim, dt=None) -> ProcessTensor:
    """ProcessTensor from ACE's PT files (layout ACE_PTB_V0): slices [0, n_init) from <name>_initial, the repeated
    slice from <name>_repeated. Raises PQDError (PQD_ERR_UNSUPPORTED) for another layout, ValueError when a file
    is missing."""
    L = _lib.lib()
    nm = str(name).encode()
    sh = _lib.pqd_ace_pt_dims()
    _lib.check(L.pqd_ace_pt_shape(nm, int(dim), sh))
    S, D, chi = sh.n_slices, sh.D, sh.chi
    Q = np.zeros((S, D, chi, chi), dtype=np.complex128)
    cl = np.zeros((S, chi), dtype=np.complex128)
    c0 = np.zeros(chi, dtype=np.complex128)
    b0 = np.zeros(chi, dtype=np.complex128)
    gmap = np.zeros(dim * dim, dtype=np.int32)
    _lib.check(L.pqd_ace_pt_read(nm, int(dim), sh, _lib.cptr(Q), _lib.cptr(cl), _lib.cptr(c0), _lib.cptr(b0),
                                 _lib.iptr(gmap)))
    return ProcessTensor(Q=Q, closure=cl, closure0=c0, bond0=b0, gmap=gmap, n_init=sh.n_init, dt=dt)


def _element(M, closure, gmap):
    D, chl, chr_ = M.shape
    head = b"PTE0" + struct.pack("<2i", len(gmap), D) + np.asarray(gmap, "<i4").tobytes() + struct.pack("<2i", chl, chr_)
    return head + np.ascontiguousarray(M, "<c16").tobytes() + np.ascontiguousarray(closure, "<c16").tobytes()


def _buffer(path, elems):
    with open(path, "w") as f:
        f.write(f"ACE_PTB_V0\nelements {len(elems)}\nblocks 1\n")
    with open(path + "_0", "wb") as f:
        for e in elems:
            f.write(e)


def write_ace_pt(name, pt: ProcessTensor, bonds=None):
    """Write `pt` in layout ACE_PTB_V0 (the four files of general_system.py:194). The schedule must be ACE's: the
    slices after n_init are one repeated slice. `bonds` (optional, length n_slices + 1) gives each element's true
    bond dimensions (a PT grown from bond 1); the matrices are cut to them, which the reader pads back."""
    S = pt.n_slices
    if S != pt.n_init + 1:
        raise ValueError("ACE's layout holds n_init initial slices and ONE repeated slice")
    chi = pt.chi
    bonds = [chi] * (S + 1) if bonds is None else list(bonds)
    if bonds[S] != bonds[S - 1]:
        raise ValueError("the repeated slice must be square in the bond")
    els = []
    for s in range(S):
        bl, br = bonds[s], bonds[s + 1] if s < S - 1 else bonds[s]
        els.append(_element(pt.Q[s][:, :bl, :br], pt.closure[s][:br], pt.gmap))
    _buffer(str(name) + "_initial", els[:-1])
    _buffer(str(name) + "_repeated", els[-1:])
