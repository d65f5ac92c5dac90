"""Numerical experiment behind the minimum-norm fit: for rank-deficient x4_q
(nip above the numerical rank, the toy cases and the reference demo's c0 = 40,
fftisdf.py:461), compare J/K of several pseudo-solves against the gelsy oracle (fftisdf.py:108)
and the exact FFT-grid J/K.  CPU only.

  python tests/experiments/min_norm_fit.py toy331 [toy222 ...]

  basic    pivoted Cholesky x4[P,P] = L L^H, z[P1] = L11^-H L11^-1 y[P1], z[P2] = 0 (the round-1
           GPU fit; gelsy's QRCP without the RZ step)
  minnorm  same factor, minimum-norm solution z = L^+H L^+ y with L^+ = L11^-1 S^-1 [I  B^H],
           B = L21 L11^-1, S = I + B^H B (the complete orthogonal step, SVD-free)
  eigh     x4 = V diag(l) V^H, z = V_r diag(1/l_r) V_r^H y, l_r > cut * l_max
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE)]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402
from scipy.linalg import lapack  # noqa: E402

from cases import inputs, oracle  # noqa: E402
from oracle import isdf_ref as R, exact_ref as E  # noqa: E402


def pchol(x4, tol_rel):
    n = len(x4)
    c, piv, rank, info = lapack.zpstrf(np.array(x4, order="F"), tol=tol_rel * abs(np.diag(x4)).max(),
                                       lower=True)
    L = np.tril(c)[:, :rank]
    return L, piv - 1, rank


def w_basic(x4, yh, tol):
    L, P, r = pchol(x4, tol)
    L11 = L[:r]
    U = sl.solve_triangular(L11, yh[P[:r]], lower=True)
    G = U @ U.conj().T
    T = sl.solve_triangular(L11.conj().T, G, lower=False)
    Wpp = sl.solve_triangular(L11.conj().T, T.conj().T, lower=False).conj().T
    W = np.zeros_like(x4)
    W[np.ix_(P[:r], P[:r])] = Wpp
    return W, r


def lplus(x4, tol):
    L, P, r = pchol(x4, tol)
    L11, L21 = L[:r], L[r:]
    B = sl.solve_triangular(L11.T, L21.T, lower=False).T          # B = L21 L11^-1
    S = np.eye(r) + B.conj().T @ B
    EH = np.concatenate([np.eye(r), B.conj().T], axis=1)          # [I  B^H]  (r x nip)
    T = sl.solve_triangular(L11, sl.cho_solve(sl.cho_factor(S, lower=True), EH), lower=True)
    return T, P, r


def w_minnorm(x4, yh, tol):
    T, P, r = lplus(x4, tol)
    U = T @ yh[P]
    G = U @ U.conj().T
    Wpp = T.conj().T @ G @ T
    W = np.zeros_like(x4)
    W[np.ix_(P, P)] = Wpp
    return W, r


def w_eigh(x4, yh, cut):
    lam, V = np.linalg.eigh(x4)
    keep = lam > cut * lam.max()
    Vr, lr = V[:, keep], lam[keep]
    U = (Vr.conj().T @ yh) / lr[:, None]
    return Vr @ (U @ U.conj().T) @ Vr.conj().T, int(keep.sum())


def run(name):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    mesh = cell.mesh
    vol = abs(np.linalg.det(cell.a))
    N = coords.shape[0]
    Gv = R.get_Gv(cell.a, mesh)
    ex_j = E.exact_j(chi, dm, cell.a, mesh)
    ex_k = E.exact_k(chi, dm, cell.a, mesh, kpts, coords)
    print(f"{name}: nip {o['nip']} gelsy ranks {o['ranks']}  gelsy vs exact "
          f"dJ {abs(o['vj'] - ex_j).max():.2e} dK {abs(o['vk'] - ex_k).max():.2e}")
    variants = [("basic", w_basic, 1e-14), ("minnorm", w_minnorm, 1e-14),
                ("minnorm", w_minnorm, 1e-15), ("minnorm", w_minnorm, 1e-16),
                ("eigh", w_eigh, 1e-15), ("eigh", w_eigh, 2.2e-16)]
    for vname, fn, tol in variants:
        ws, rs = [], []
        for q, vq in enumerate(kpts):
            fq = np.exp(-1j * coords @ vq)
            cg = R.get_coulG(cell.a, vq, mesh, Gv=Gv) * vol / N / N
            yh = R.fft(o["y"][q].T * fq, mesh) * np.sqrt(cg)
            w, r = fn(o["x4"][q], yh, tol)
            ws.append(w)
            rs.append(r)
        w = np.asarray(ws)
        vj = R.get_j_kpts(o["xip"], w[0], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
        vk = R.get_k_kpts(o["xip"], w, dm, phase)
        print(f"  {vname:8s} tol {tol:.1e} ranks {min(rs)}-{max(rs)}: vs gelsy dJ "
              f"{abs(vj - o['vj']).max():.2e} dK {abs(vk - o['vk']).max():.2e} | vs exact dJ "
              f"{abs(vj - ex_j).max():.2e} dK {abs(vk - ex_k).max():.2e}", flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["toy331", "toy222"]:
        run(n)


def w_cod(x4, yh, tol):
    """minimum-norm solution from the pivoted Cholesky via a thin QR of A = P L (nip x r):
    x4 ~ A A^H, z = A^{+H} A^+ y, A^+ = R_A^{-1} Q_A^H (no normal equations)."""
    L, P, r = pchol(x4, tol)
    A = np.zeros((len(x4), r), complex)
    A[P] = L
    Qa, Ra = np.linalg.qr(A)
    M = sl.solve_triangular(Ra, Qa.conj().T)          # r x nip  = A^+
    U = M @ yh
    G = U @ U.conj().T
    return M.conj().T @ G @ M, r


if __name__ == "__main__" and os.environ.get("COD"):
    pass
