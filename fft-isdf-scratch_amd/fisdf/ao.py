"""Bloch AO values on the GPU: the input layer PySCF's
``pbc_eval_gto('GTOval', coords, kpts)`` provides to ``fftisdf.py:72,367-370``.

``eval_ao_kpts_gpu`` returns the same array as ``cell.eval_ao_kpts`` (the host restatement),
computed by ``fisdf_eval_ao`` (csrc/ao.hip) and left resident on the device."""
from __future__ import annotations

import numpy as np

from . import _lib
from .cell import cell_rcut, lattice_translations


def _shell_tables(cell):
    sh_atom, sh_l, sh_np, exps, coefs = [], [], [], [], []
    for (ia, l, e, c, _ao0) in cell.shells:
        sh_atom.append(ia)
        sh_l.append(l)
        sh_np.append(len(e))
        exps.extend(np.asarray(e, float).tolist())
        coefs.extend(np.asarray(c, float).tolist())
    return (np.asarray(sh_atom, np.int32), np.asarray(sh_l, np.int32), np.asarray(sh_np, np.int32),
            np.asarray(exps, np.float64), np.asarray(coefs, np.float64))


def eval_ao_band_gpu(device, cell, coords, kpts):
    """chi_k(r) at arbitrary k-points ``kpts`` (nkb, 3) (``fisdf_eval_ao_band``; host
    restatement ``cell.eval_ao_band``): device tensor (nkb, ng, nao)."""
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    kpts = np.ascontiguousarray(np.asarray(kpts, float).reshape(-1, 3))
    ng, nao = coords.shape[0], cell.nao_nr()
    tn = np.ascontiguousarray(lattice_translations(cell, coords), dtype=np.int32)
    sh_atom, sh_l, sh_np, exps, coefs = _shell_tables(cell)
    atoms = np.ascontiguousarray(cell.atom_coords(), dtype=np.float64)
    dcoords = device.torch.as_tensor(coords, device=device.dev)
    out = device.empty((len(kpts), ng, nao))
    a, ap = _lib.darr(np.asarray(cell.lattice_vectors(), float).ravel())
    ip, dp = _lib._ip, _lib._dp
    device.ctx.call("fisdf_eval_ao_band", _lib.ptr(dcoords), ng, len(atoms),
                    atoms.ctypes.data_as(dp), len(sh_l), sh_atom.ctypes.data_as(ip),
                    sh_l.ctypes.data_as(ip), sh_np.ctypes.data_as(ip), exps.ctypes.data_as(dp),
                    coefs.ctypes.data_as(dp), len(tn), tn.ctypes.data_as(ip), len(kpts),
                    kpts.ctypes.data_as(dp), ap, cell_rcut(cell), nao, _lib.ptr(out))
    return out


def eval_ao_kpts_gpu(device, cell, coords, kmesh):
    """chi_k(r) for the k-mesh ``kmesh`` at ``coords`` (ng, 3): device tensor (nk, ng, nao)."""
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    ng = coords.shape[0]
    kmesh = [int(k) for k in kmesh]
    nk = int(np.prod(kmesh))
    nao = cell.nao_nr()
    tn = np.ascontiguousarray(lattice_translations(cell, coords), dtype=np.int32)
    sh_atom, sh_l, sh_np, exps, coefs = [], [], [], [], []
    for (ia, l, e, c, _ao0) in cell.shells:
        sh_atom.append(ia)
        sh_l.append(l)
        sh_np.append(len(e))
        exps.extend(np.asarray(e, float).tolist())
        coefs.extend(np.asarray(c, float).tolist())
    sh_atom = np.asarray(sh_atom, np.int32)
    sh_l = np.asarray(sh_l, np.int32)
    sh_np = np.asarray(sh_np, np.int32)
    exps = np.asarray(exps, np.float64)
    coefs = np.asarray(coefs, np.float64)
    atoms = np.ascontiguousarray(cell.atom_coords(), dtype=np.float64)
    torch = device.torch
    dcoords = torch.as_tensor(coords, device=device.dev)
    out = device.empty((nk, ng, nao))
    km, kmp = _lib.iarr(kmesh)
    a, ap = _lib.darr(np.asarray(cell.lattice_vectors(), float).ravel())
    ip, dp = _lib._ip, _lib._dp
    device.ctx.call("fisdf_eval_ao", _lib.ptr(dcoords), ng, len(atoms),
                    atoms.ctypes.data_as(dp), len(sh_l), sh_atom.ctypes.data_as(ip),
                    sh_l.ctypes.data_as(ip), sh_np.ctypes.data_as(ip), exps.ctypes.data_as(dp),
                    coefs.ctypes.data_as(dp), len(tn), tn.ctypes.data_as(ip), kmp, ap,
                    cell_rcut(cell), nao, _lib.ptr(out))
    return out
