"""Which rank decision puts the minimum-norm fit closest to gelsy (fftisdf.py:108)
in the reference demo's regime (C2, c0 = 1e4 -> nip = parent rank, every x4_q rank-deficient)?
gelsy ranks x4_q by QRCP + an incremental condition estimate at rcond = eps; the GPU's fit ranks
it by a pivoted-Cholesky cut d_r <= tol * max diag.  For each q this prints gelsy's rank beside
the Cholesky cuts and a condition-number rule on the Cholesky factor, then J/K of the min-norm fit
at (a) gelsy's own per-q rank and (b) each rule, against gelsy at its default rcond.  CPU only.

  python tests/experiments/rank_rule_c2.py
  python tests/experiments/rank_rule_c2.py --gpu OUT.npz   (tools/rank_regime_gpu.py's builds)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE), HERE]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402
from scipy.linalg import lapack  # noqa: E402

import bench  # noqa: E402
from oracle import isdf_ref as R  # noqa: E402

EPS = np.finfo(float).eps


def gelsy_rank(a, rcond):
    b = np.ones((len(a), 1), complex)
    n = len(a)
    work, _ = lapack.zgelsy_lwork(n, n, 1, rcond)
    out = lapack.zgelsy(np.array(a, order="F"), b, np.zeros(n, np.int32), rcond, int(work.real))
    return int(out[3])


def pchol_full(x4, tol_rel=1e-18):
    c, piv, rank, info = lapack.zpstrf(np.array(x4, order="F"), tol=tol_rel * abs(np.diag(x4)).max(),
                                       lower=True)
    return np.tril(c)[:, :rank], piv - 1, rank


def cod_w(L, P, r, yh):
    A = np.zeros((L.shape[0], r), complex)
    A[P] = L[:, :r]
    Qa, Ra = np.linalg.qr(A)
    M = sl.solve_triangular(Ra, Qa.conj().T)
    U = M @ yh
    return M.conj().T @ (U @ U.conj().T) @ M


def cond_rank(L, bound, lo, hi):
    """largest r in [lo, hi] with cond(L[:r,:r])^2 <= bound (cond by SVD, bisection; cond of a
    growing leading block is monotone)"""
    def ok(r):
        s = np.linalg.svd(L[:r, :r], compute_uv=False)
        return (s[0] / s[-1]) ** 2 <= bound
    if not ok(lo):
        return lo
    while hi - lo > 1:
        mid = (lo + hi) // 2
        lo, hi = (mid, hi) if ok(mid) else (lo, mid)
    return lo


def gpu_compare(path):
    """J/K of GPU builds at several fit_tol cuts (tools/rank_regime_gpu.py) against gelsy at its
    default rcond and gelsy's own rcond band (4 eps, eps / 4), on the GPU's points."""
    g = dict(np.load(path))
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c2")
    dms = dm[None]
    perm = g["perm"]
    xip = x0[:, perm]
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    x4 = R.build_x4(xip, phase)
    coords = cell.gen_uniform_grids(cell.mesh)
    mesh, vol, N = cell.mesh, cell.vol, coords.shape[0]
    Gv = R.get_Gv(cell.a, mesh)
    y_all = np.empty((len(kpts), N, len(perm)), complex)
    for g0 in range(0, N, 8000):
        y_all[:, g0:g0 + 8000] = R.build_y(chi[:, g0:g0 + 8000], xip, phase)
    res = {}
    for tag, cond in (("gelsy", None), ("gelsy x4", 4 * EPS), ("gelsy /4", EPS / 4)):
        ws, rs = [], []
        for q, vq in enumerate(kpts):
            fq = np.exp(-1j * coords @ vq)
            z, _, r, _ = sl.lstsq(x4[q], y_all[q].T, cond=cond, lapack_driver="gelsy")
            zeta = R.fft(z * fq, mesh) * R.get_coulG(cell.a, vq, mesh, Gv=Gv) * (vol / N)
            ws.append((R.ifft(zeta, mesh) * fq.conj()) @ z.conj().T)
            rs.append(r)
        w = np.asarray(ws)
        res[tag] = (R.get_j_kpts(xip, w[0], dms)[0], R.get_k_kpts(xip, w, dms, phase)[0], rs)
        print(f"  {tag:9s} ranks {rs}", flush=True)
    vj0, vk0, _ = res["gelsy"]
    bj = max(abs(res[t][0] - vj0).max() for t in ("gelsy x4", "gelsy /4"))
    bk = max(abs(res[t][1] - vk0).max() for t in ("gelsy x4", "gelsy /4"))
    print(f"  gelsy's own rcond band |dJ| {bj:.2e} |dK| {bk:.2e}  (nip {len(perm)})")
    for tol in g["tols"]:
        tag = f"{tol:.1e}"
        ej = abs(g[f"vj_{tag}"] - vj0).max()
        ek = abs(g[f"vk_{tag}"] - vk0).max()
        print(f"  GPU fit_tol {tag} ranks {g[f'ranks_{tag}'].tolist()}: vs gelsy |dJ| {ej:.2e} "
              f"({ej / bj:.2f} band) |dK| {ek:.2e} ({ek / bk:.2f} band)", flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--gpu":
        return gpu_compare(sys.argv[2])
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c2")
    dms = dm[None]
    perm, rank, nip, _ = R.select_interpolation_points(x0, cell.nao_nr(), 1e4)
    xip = x0[:, perm]
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    x4 = R.build_x4(xip, phase)
    coords = cell.gen_uniform_grids(cell.mesh)
    mesh, vol, N = cell.mesh, cell.vol, coords.shape[0]
    Gv = R.get_Gv(cell.a, mesh)
    print(f"c2 rank regime: nip {nip}", flush=True)
    facs, rows = [], []
    for q in range(len(kpts)):
        L, P, rmax = pchol_full(x4[q])
        d = np.abs(np.diag(L)) ** 2
        rg = gelsy_rank(x4[q], EPS)
        cuts = {t: int(np.sum(d > t * d[0])) for t in (1e-14, 3e-15, 1e-15, 3e-16)}
        rc = cond_rank(L, 1 / EPS, min(cuts.values()) - 50, min(rmax, max(cuts.values()) + 50))
        facs.append((L, P))
        rows.append((rg, cuts, rc))
        print(f"  q{q}: gelsy {rg}  chol cuts {cuts}  cond(L11)^2<=1/eps {rc}  (factor {rmax})",
              flush=True)
    y_all = np.empty((len(kpts), N, nip), complex)
    for g0 in range(0, N, 8000):
        g1 = min(g0 + 8000, N)
        y_all[:, g0:g1] = R.build_y(chi[:, g0:g1], xip, phase)
    yh = []
    for q, vq in enumerate(kpts):
        fq = np.exp(-1j * coords @ vq)
        cg = R.get_coulG(cell.a, vq, mesh, Gv=Gv) * vol / N / N
        yh.append(R.fft(y_all[q].T * fq, mesh) * np.sqrt(cg))
    t = time.perf_counter()
    ws = []
    for q, vq in enumerate(kpts):
        fq = np.exp(-1j * coords @ vq)
        z, _, r, _ = sl.lstsq(x4[q], y_all[q].T, lapack_driver="gelsy")
        zeta = R.fft(z * fq, mesh) * R.get_coulG(cell.a, vq, mesh, Gv=Gv) * (vol / N)
        ws.append((R.ifft(zeta, mesh) * fq.conj()) @ z.conj().T)
    w = np.asarray(ws)
    vj0, vk0 = R.get_j_kpts(xip, w[0], dms), R.get_k_kpts(xip, w, dms, phase)
    print(f"  gelsy done ({time.perf_counter() - t:.0f} s)", flush=True)
    rules = {"gelsy rank": [r[0] for r in rows], "cond rule": [r[2] for r in rows]}
    for tcut in (1e-14, 3e-15, 1e-15):
        rules[f"chol {tcut:.0e}"] = [r[1][tcut] for r in rows]
    for tag, ranks in rules.items():
        w = np.asarray([cod_w(L, P, r, yh[q]) for q, ((L, P), r) in enumerate(zip(facs, ranks))])
        vj, vk = R.get_j_kpts(xip, w[0], dms), R.get_k_kpts(xip, w, dms, phase)
        print(f"  min-norm at {tag:11s} ranks {min(ranks)}-{max(ranks)}: vs gelsy |dJ| "
              f"{abs(vj - vj0).max():.2e} |dK| {abs(vk - vk0).max():.2e}", flush=True)


if __name__ == "__main__":
    main()
