"""How much do the reference's own J/K depend on its selection's tie-breaking?  (VERDICT r02
"next round" item 1; run on the CPU, no GPU.)

The parent-grid Gram x4 of a symmetric crystal has exactly tied diagonal entries (symmetry-
equivalent grid points), so LAPACK dpstrf's greedy pivots are decided by the last bits of x2 —
i.e. by the BLAS's summation order.  Here the oracle (fftisdf.py:357-388 + :22-228) is run on
the same cell and k-mesh with x2 formed in two equally valid orders:
  A: sum_q Re(conj(x0_q) x0_q^T)        (fftisdf.py:376-378, the oracle's order)
  B: Re parts split, Xr Xr^T + Xi Xi^T with all q stacked (one GEMM, another order)
and both builds' J/K are compared with each other and with the exact FFT-grid J/K.

  python tests/experiments/selection_sensitivity.py [c2|toy222|...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.join(ROOT, "tests")]

from oracle import isdf_ref as R  # noqa: E402
from oracle import exact_ref as E  # noqa: E402


def inputs(cfg):
    if cfg.startswith("c"):
        import bench
        cell, kmesh, m0, c0, x0, chi, dm = bench.setup(cfg)
        return cell, kmesh, c0, x0, chi, dm[None]
    from cases import inputs as ci
    cell, kmesh, m0, c0, x0, coords, chi, dm = ci(cfg)
    return cell, kmesh, c0, x0, chi, dm


def select_from(x2, nao, c0, nk):
    x4 = x2 * x2 / nk
    _, perm, rank = R.pivoted_cholesky(x4)
    nip = min(int(nao * c0), rank)
    return perm[:nip], rank


def jk(cell, kmesh, x0, chi, dm, perm):
    xip = x0[:, perm]
    coords = cell.gen_uniform_grids(cell.mesh)
    out = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    vj = R.get_j_kpts(xip, out["w0"], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk = R.get_k_kpts(xip, out["wq"], dm, phase)
    return vj, vk


def main(cfg="c2"):
    cell, kmesh, c0, x0, chi, dm = inputs(cfg)
    nk, ng0, nao = x0.shape
    t = time.perf_counter()
    x2a = np.zeros((ng0, ng0))
    for q in range(nk):
        x2a += (x0[q].conj() @ x0[q].T).real
    P = x0.transpose(1, 0, 2).reshape(ng0, nk * nao)
    x2b = P.real @ P.real.T + P.imag @ P.imag.T
    print(f"{cfg}: nk {nk} ng0 {ng0} nao {nao}; max |x2a - x2b| / max|x2a| "
          f"{abs(x2a - x2b).max() / abs(x2a).max():.1e}", flush=True)
    pa, ra = select_from(x2a, nao, c0, nk)
    pb, rb = select_from(x2b, nao, c0, nk)
    first = next((i for i in range(min(len(pa), len(pb))) if pa[i] != pb[i]), None)
    shared = len(set(pa) & set(pb)) / len(pa)
    print(f"  rank {ra} / {rb}, nip {len(pa)}; first divergence at pivot {first}, shared points "
          f"{100 * shared:.0f}%  ({time.perf_counter() - t:.1f} s)", flush=True)
    t = time.perf_counter()
    vja, vka = jk(cell, kmesh, x0, chi, dm, pa)
    vjb, vkb = jk(cell, kmesh, x0, chi, dm, pb)
    print(f"  J/K between the two selections: |dJ| {abs(vja - vjb).max():.2e} "
          f"|dK| {abs(vka - vkb).max():.2e}  ({time.perf_counter() - t:.1f} s)", flush=True)
    t = time.perf_counter()
    kpts = R.get_kpts(cell.a, kmesh)
    coords = cell.gen_uniform_grids(cell.mesh)
    vje = E.exact_j(chi, dm, cell.a, cell.mesh)
    vke = E.exact_k(chi, dm, cell.a, cell.mesh, kpts, coords)
    if abs(kpts).max() < 1e-9:
        vje = vje.real
    for tag, vj, vk in (("A", vja, vka), ("B", vjb, vkb)):
        print(f"  selection {tag} vs exact FFT-grid: |dJ| {abs(vj - vje).max():.2e} "
              f"|dK| {abs(vk - vke).max():.2e}", flush=True)
    print(f"  (exact J/K {time.perf_counter() - t:.1f} s; max|J| {abs(vje).max():.3f} "
          f"max|K| {abs(vke).max():.3f})")


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["c2"]))
