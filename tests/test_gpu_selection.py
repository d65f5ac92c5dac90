"""Interpolation-point selection (fftisdf.py:357-388) on the GPU vs LAPACK dpstrf at the real
m0 = 15^3 parent grids of every BASELINE config (C1-C5) and the toy cases.

Greedy full pivoting on a symmetric crystal meets exact ties (symmetry-equivalent points) that
only rounding breaks, and dpstrf's rounding (blocked, OpenBLAS dsyrk trailing updates) cannot
be reproduced bit for bit.  So the GPU pivots must equal dpstrf's, or — from the first
divergence on — carry a tie certificate computed here in float64 on the host:
  * at the first differing step p both candidates are maximal residual diagonals of the common
    prefix to within the dpstrf tolerance scale: d_p[gpu] >= max(d_p) - ng0 eps max(diag);
  * the greedy run along the GPU's order ends with the same residual as dpstrf's:
    |max res_gpu - max res_lapack| <= ng0 eps max(diag)  (same selection quality).
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def residual_along(x4, order):
    """Pivoted Cholesky of x4 along a given pivot order (float64, host): the residual diagonal
    before each step, and after the last one."""
    n = x4.shape[0]
    d = np.diag(x4).copy()
    L = np.zeros((n, len(order)))
    before = []
    for j, p in enumerate(order):
        before.append(d.copy())
        col = (x4[:, p] - L[:, :j] @ L[p, :j]) / np.sqrt(d[p])
        L[:, j] = col
        d = d - col * col
        d[order[:j + 1]] = 0.0
    return before, d


def gpu_select(x0, nao, nip_max, tol=-1.0):
    import ctypes as C
    import torch
    from fisdf import _lib as L
    ctx = L.Context(0, torch.cuda.current_stream().cuda_stream)
    dx0 = torch.from_numpy(np.ascontiguousarray(x0)).cuda()
    nk, ng0 = x0.shape[:2]
    perm = np.zeros(nip_max, np.int32)
    npiv, full = C.c_int(), C.c_int()
    ctx.call("fisdf_select_points", L.ptr(dx0), nk, ng0, nao, nip_max, tol,
             perm.ctypes.data_as(L._ip), C.byref(npiv), C.byref(full))
    ctx.close()
    return perm[:min(nip_max, npiv.value)]


def gpu_select_km(x0, kmesh, nao, nip_max, tol=-1.0, time_reversal=True):
    """fisdf_select_points_km: with time reversal the Gram is folded over the representatives
    k <= -k (fisdf_set_time_reversal)."""
    import ctypes as C
    import torch
    from fisdf import _lib as L
    ctx = L.Context(0, torch.cuda.current_stream().cuda_stream)
    ctx.call("fisdf_set_time_reversal", 1 if time_reversal else 0)
    dx0 = torch.from_numpy(np.ascontiguousarray(x0)).cuda()
    ng0 = x0.shape[1]
    perm = np.zeros(nip_max, np.int32)
    npiv, full = C.c_int(), C.c_int()
    km = (C.c_int * 3)(*[int(k) for k in kmesh])
    ctx.call("fisdf_select_points_km", L.ptr(dx0), km, ng0, nao, nip_max, tol,
             perm.ctypes.data_as(L._ip), C.byref(npiv), C.byref(full))
    ctx.close()
    return perm[:min(nip_max, npiv.value)]


def _cell_x0(cfg):
    import bench
    from fisdf import cell as C
    kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS[cfg]
    make = {"diamond": C.diamond_cell, "nio": C.nio_cell, "si": C.si_supercell}[kind]
    cell = make(basis=basis, mesh=mesh)
    c0 = (nip + 0.5) / cell.nao_nr()
    return cell, kmesh, c0, C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg", ["c1", "c2", "c3", "c4", "c5", "toy222", "toy331", "toy333_fr"])
def test_selection_vs_dpstrf(cfg):
    from oracle import isdf_ref as R
    if cfg.startswith("toy"):
        from cases import inputs
        cell, kmesh, m0, c0, x0 = inputs(cfg)[:5]
    else:
        cell, kmesh, c0, x0 = _cell_x0(cfg)
    nao = cell.nao_nr()
    perm_l, rank, nip, x4 = R.select_interpolation_points(x0, nao, c0)
    perm_g = gpu_select(x0, nao, int(nao * c0))
    ng0 = x4.shape[0]
    assert len(perm_g) == nip, (len(perm_g), nip)
    same = perm_g == perm_l
    first = int(np.argmin(same)) if not same.all() else nip
    tie_tol = ng0 * np.finfo(float).eps * np.diag(x4).max()
    msg = f"{cfg}: ng0 {ng0} rank {rank} nip {nip}: identical prefix {first}/{nip}"
    if first < nip:
        before, res_g = residual_along(x4, perm_g)
        _, res_l = residual_along(x4, perm_l)
        dp = before[first]
        gap = dp.max() - dp[perm_g[first]]
        dres = abs(res_g.max() - res_l.max())
        overlap = len(set(perm_g.tolist()) & set(perm_l.tolist())) / nip
        msg += (f"; tie at step {first}: d[gpu] {dp[perm_g[first]]:.17e} d[lapack] "
                f"{dp[perm_l[first]]:.17e} gap {gap:.1e} (tol {tie_tol:.1e}); final max residual "
                f"gpu {res_g.max():.6e} lapack {res_l.max():.6e}; set overlap {overlap:.3f}")
        print(msg)
        assert gap <= tie_tol
        assert dres <= tie_tol
    else:
        print(msg)


def _tie_certified(x4, perm_g, perm_l, what):
    nip = len(perm_l)
    assert len(perm_g) == nip, (what, len(perm_g), nip)
    same = perm_g == perm_l
    first = int(np.argmin(same)) if not same.all() else nip
    print(f"{what}: identical prefix {first}/{nip}")
    if first == nip:
        return
    tie_tol = x4.shape[0] * np.finfo(float).eps * np.diag(x4).max()
    before, res_g = residual_along(x4, perm_g)
    _, res_l = residual_along(x4, perm_l)
    dp = before[first]
    assert dp.max() - dp[perm_g[first]] <= tie_tol
    assert abs(res_g.max() - res_l.max()) <= tie_tol


@pytest.mark.timeout(300)
def test_selection_folded_gram_large_kmesh():
    """a k-mesh with more than 64 time-reversal representatives (6x6x6: 112)
    goes through the folded selection Gram in several 64-k launches; the pivots are dpstrf's
    (or tie-certified) with and without the fold."""
    from oracle import isdf_ref as R
    from cases import inputs
    cell, kmesh, m0, c0, x0 = inputs("toy666")[:5]
    nao = cell.nao_nr()
    perm_l, rank, nip, x4 = R.select_interpolation_points(x0, nao, c0)
    for tr in (True, False):
        perm_g = gpu_select_km(x0, kmesh, nao, int(nao * c0), time_reversal=tr)
        _tie_certified(x4, perm_g, perm_l, f"toy666 time_reversal={tr}")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "toy222"])
def test_selection_batch_equals_coop(cfg, monkeypatch):
    """The batched-candidate kernel (FISDF_SEL_MODE=batch; the default from 800 pivots on) and
    the cooperative one pick the same pivots — every batched step is the greedy pivot of the
    whole matrix, so the sequences agree to the last pivot (ties aside: both break them by the
    smaller row on equal values computed in the same order)."""
    if cfg.startswith("toy"):
        from cases import inputs
        cell, kmesh, m0, c0, x0 = inputs(cfg)[:5]
    else:
        cell, kmesh, c0, x0 = _cell_x0(cfg)
    nao = cell.nao_nr()
    perms = {}
    for mode in ("coop", "batch"):
        monkeypatch.setenv("FISDF_SEL_MODE", mode)
        perms[mode] = gpu_select(x0, nao, int(nao * c0))
    same = perms["coop"] == perms["batch"]
    print(f"{cfg}: coop {len(perms['coop'])} batch {len(perms['batch'])} pivots, identical "
          f"{int(same.sum()) if len(same) else 0}")
    assert np.array_equal(perms["coop"], perms["batch"])
