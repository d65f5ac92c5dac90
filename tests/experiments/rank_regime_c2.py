"""The reference demo's regime at full size (fftisdf.py:455-461: nip reaches the parent-Gram
rank, every x4_q rank-deficient), C2's cell / mesh / k-mesh, CPU only: how far do J/K move
between gelsy (fftisdf.py:108) at its default rcond and gelsy at 4x / 0.25x that rcond, and how
far does the minimum-norm fit of the GPU (pivoted Cholesky, thin QR of P L) sit
from gelsy at each Cholesky rank cut.  Points: dpstrf's (c0 = 1e4 -> nip = rank).

  python tests/experiments/rank_regime_c2.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE), HERE]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402

import bench  # noqa: E402
from min_norm_fit import w_cod  # noqa: E402
from oracle import isdf_ref as R  # noqa: E402


def main():
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c2")
    dms = dm[None]
    t = time.perf_counter()
    perm, rank, nip, _ = R.select_interpolation_points(x0, cell.nao_nr(), 1e4)
    xip = x0[:, perm]
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    x4 = R.build_x4(xip, phase)
    coords = cell.gen_uniform_grids(cell.mesh)
    mesh, vol, N = cell.mesh, cell.vol, coords.shape[0]
    Gv = R.get_Gv(cell.a, mesh)
    print(f"c2 rank regime: nip {nip} = parent rank {rank}  ({time.perf_counter() - t:.1f} s)",
          flush=True)
    y_all = np.empty((len(kpts), N, nip), complex)
    for g0 in range(0, N, 8000):
        g1 = min(g0 + 8000, N)
        y_all[:, g0:g1] = R.build_y(chi[:, g0:g1], xip, phase)
    eps = np.finfo(float).eps
    res = {}
    for tag, cond in (("gelsy", None), ("gelsy x4", 4 * eps), ("gelsy /4", eps / 4)):
        t = time.perf_counter()
        ws, rs = [], []
        for q, vq in enumerate(kpts):
            fq = np.exp(-1j * coords @ vq)
            z, _, r, _ = sl.lstsq(x4[q], y_all[q].T, cond=cond, lapack_driver="gelsy")
            zeta = R.fft(z * fq, mesh) * R.get_coulG(cell.a, vq, mesh, Gv=Gv) * (vol / N)
            zeta = R.ifft(zeta, mesh) * fq.conj()
            ws.append(zeta @ z.conj().T)
            rs.append(r)
        w = np.asarray(ws)
        res[tag] = (R.get_j_kpts(xip, w[0], dms), R.get_k_kpts(xip, w, dms, phase))
        print(f"  {tag:9s} ranks {min(rs)}-{max(rs)} ({time.perf_counter() - t:.0f} s)", flush=True)
    for tol in (1e-14, 1e-15, 2.2e-16):
        t = time.perf_counter()
        ws, rs = [], []
        for q, vq in enumerate(kpts):
            fq = np.exp(-1j * coords @ vq)
            cg = R.get_coulG(cell.a, vq, mesh, Gv=Gv) * vol / N / N
            w, r = w_cod(x4[q], R.fft(y_all[q].T * fq, mesh) * np.sqrt(cg), tol)
            ws.append(w)
            rs.append(r)
        w = np.asarray(ws)
        res[f"cod {tol:.0e}"] = (R.get_j_kpts(xip, w[0], dms), R.get_k_kpts(xip, w, dms, phase))
        print(f"  cod tol {tol:.1e} ranks {min(rs)}-{max(rs)} ({time.perf_counter() - t:.0f} s)",
              flush=True)
    vj0, vk0 = res["gelsy"]
    for tag, (vj, vk) in res.items():
        print(f"  {tag:12s} vs gelsy(rcond eps): |dJ| {abs(vj - vj0).max():.2e} "
              f"|dK| {abs(vk - vk0).max():.2e}", flush=True)


if __name__ == "__main__":
    main()
