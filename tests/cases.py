"""Shared small cases for CPU and GPU tests (inputs are regenerated deterministically)."""
import functools

import numpy as np

from fisdf import cell as C
from oracle import isdf_ref as R


CASES = {
    # name: (cell factory, kmesh, m0, c0)
    "toy222": (lambda: C.toy_cell(mesh=(12, 12, 12)), (2, 2, 2), (9, 9, 9), 40.0),
    "toy331": (lambda: C.toy_cell(mesh=(15, 15, 15)), (3, 3, 1), (9, 9, 9), 40.0),
    # production regime: nip below the numerical rank, every x4_q full rank (as at C2/C3,
    # ranks == nip); the toy cases above have nip > rank (x4_q rank-deficient)
    "toy331_fr": (lambda: C.toy_cell(mesh=(15, 15, 15)), (3, 3, 1), (9, 9, 9), 25.0),
    "toy333_fr": (lambda: C.toy_cell(mesh=(12, 12, 12)), (3, 3, 3), (9, 9, 9), 20.0),
    "diamond_szv_gamma": (lambda: C.diamond_cell(basis="gth-szv", mesh=(8, 8, 8)), (1, 1, 1),
                          (15, 15, 15), 20.0),
    # C4-shaped: NiO AFM (nio-afm.vasp), dzvp-molopt-sr-shaped basis with f shells (nao 76);
    # reduced mesh/k-mesh so the gelsy oracle runs in seconds
    "nio_small": (lambda: C.nio_cell(mesh=(16, 16, 16)), (1, 1, 2), (9, 9, 9), 5.0),
    # C5-shaped: Si 2x2x2 diamond supercell, 16 atoms, szv-shaped (nao 64), Gamma only
    "si_small": (lambda: C.si_supercell(mesh=(12, 12, 12)), (1, 1, 1), (9, 9, 9), 8.0),
    # the reference demo's regime (fftisdf.py:455-461, c0 = 40 with m0 = 15^3): nao * c0
    # exceeds the parent-Gram rank, so nip = rank (fftisdf.py:383) and every x4_q is
    # rank-deficient
    "toy222_rank": (lambda: C.toy_cell(mesh=(12, 12, 12)), (2, 2, 2), (9, 9, 9), 100.0),
    # a k-mesh with more time-reversal representatives (112) than one kernel argument block
    # holds (64): the folded selection Gram, x4 and y take their multi-launch / generic paths
    "toy666": (lambda: C.toy_cell(mesh=(10, 10, 10)), (6, 6, 6), (7, 7, 7), 5.0),
}


@functools.lru_cache(maxsize=None)
def inputs(name):
    make, kmesh, m0, c0 = CASES[name]
    cell = make()
    x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
    coords = cell.gen_uniform_grids(cell.mesh)
    chi = C.eval_ao_kpts(cell, coords, kmesh)
    dm = C.make_dm(cell.nao_nr(), kmesh, cell, seed=1234)[None]
    return cell, kmesh, m0, c0, x0, coords, chi, dm


@functools.lru_cache(maxsize=None)
def oracle_y(name):
    """Selection + y only (no fit): cheap enough for the spawned multi-rank workers."""
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    perm, rank, nip, _ = R.select_interpolation_points(x0, cell.nao_nr(), c0)
    xip = x0[:, perm, :]
    phase = R.get_phase(cell.a, R.get_kpts(cell.a, kmesh), kmesh)
    return dict(perm=perm, xip=xip, y=R.build_y(chi, xip, phase))


@functools.lru_cache(maxsize=None)
def oracle(name):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    perm, rank, nip, x4sel = R.select_interpolation_points(x0, cell.nao_nr(), c0)
    xip = x0[:, perm, :]
    out = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    # fftisdf.py:169-170: vj.real when the k-points are all zero (Gamma-only runs)
    vj = R.get_j_kpts(xip, out["w0"], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk = R.get_k_kpts(xip, out["wq"], dm, phase)
    return dict(perm=perm, rank=rank, nip=nip, x4sel=x4sel, xip=xip, vj=vj, vk=vk, **out)


@functools.lru_cache(maxsize=None)
def oracle_svd(name):
    """The oracle with the SVD pseudo-solve (fftdf-with-k-svd.py:158-164 intent) on the gelsy
    oracle's interpolation points."""
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    out = R.build(o["xip"], chi, coords, cell.a, kmesh, cell.mesh, solver="svd")
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    vj = R.get_j_kpts(o["xip"], out["w0"], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk = R.get_k_kpts(o["xip"], out["wq"], dm, phase)
    return dict(vj=vj, vk=vk, ranks=out["ranks"], wq=out["wq"])
