"""Can the fit's Coulomb HERK G = U U^H (U = L^-1 Yhat, weights folded in) run as
an int8 Ozaki-scheme emulation and keep J/K at the FP64 path's accuracy?  CPU only.

  python tests/experiments/ozaki_herk.py toy331_fr [toy333_fr ...]

Each row of Re U and Im U is scaled by a power of two (its max) and split into S signed 7-bit
digit slices; Re G = Ur Ur^T + Ui Ui^T and Im G = Ui Ur^T - Ur Ui^T are formed from the slice
products with s + t <= S + 1 (exact here: integer digits in float64 stay below 2^53; int32 MFMA
accumulation over K chunks on the device), and J/K are compared with the FP64 HERK.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE)]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402

from cases import inputs, oracle  # noqa: E402
from oracle import isdf_ref as R  # noqa: E402


def slices(X, S, bits=7):
    """X (rows x K) real -> (exponent per row, S int8 digit slices) with X ~ sum_s d_s 2^(e - bits s)."""
    m = np.abs(X).max(axis=1)
    e = np.where(m > 0, np.ceil(np.log2(np.where(m > 0, m, 1.0))), 0.0)
    r = X / 2.0 ** e[:, None]                      # |r| <= 1
    out = []
    for _ in range(S):
        r = r * 2 ** bits
        d = np.rint(r)
        out.append(d)       # integer-valued float64: the products are exact below 2^53
        r = r - d
    return e, out


def oz_product(A, B, S, bits=7):
    """A B^T from the slice products with s + t <= S + 1 (A, B real, rows x K)."""
    ea, sa = slices(A, S, bits)
    eb, sb = slices(B, S, bits)
    P = np.zeros((A.shape[0], B.shape[0]))
    for s in range(S):
        for t in range(S - s):
            P += (sa[s] @ sb[t].T) * 2.0 ** (-bits * (s + t + 2))
    return P * 2.0 ** ea[:, None] * 2.0 ** eb[None, :]


def herk_oz(U, S):
    Ur, Ui = U.real, U.imag
    Gr = oz_product(Ur, Ur, S) + oz_product(Ui, Ui, S)
    Gi = oz_product(Ui, Ur, S) - oz_product(Ur, Ui, S)
    return Gr + 1j * Gi


def run(name, Ss=(4, 5, 6)):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    vol = abs(np.linalg.det(cell.a))
    N = coords.shape[0]
    Gv = R.get_Gv(cell.a, cell.mesh)
    res = {S: [] for S in (0,) + tuple(Ss)}
    for q, vq in enumerate(kpts):
        fq = np.exp(-1j * coords @ vq)
        cg = R.get_coulG(cell.a, vq, cell.mesh, Gv=Gv) * vol / N / N
        yh = R.fft(o["y"][q].T * fq, cell.mesh) * np.sqrt(cg)
        L = np.linalg.cholesky(o["x4"][q])
        U = sl.solve_triangular(L, yh, lower=True)
        for S in res:
            G = U @ U.conj().T if S == 0 else herk_oz(U, S)
            T = sl.solve_triangular(L.conj().T, G, lower=False)
            res[S].append(sl.solve_triangular(L.conj().T, T.conj().T, lower=False).conj().T)
    for S, ws in res.items():
        w = np.asarray(ws)
        vj = R.get_j_kpts(o["xip"], w[0], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
        vk = R.get_k_kpts(o["xip"], w, dm, phase)
        print(f"{name} S={S} ({7 * S} bits): vs gelsy dJ {abs(vj - o['vj']).max():.2e} "
              f"dK {abs(vk - o['vk']).max():.2e}", flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["toy331_fr"]:
        run(n)
