"""Numerical experiment behind the 3-multiplication complex GEMM: the fit's
TRSM (U = L^{-1} Yhat, explicit triangular inverse) and HERK (U D U^H) formed with
Re = P1 - P2, Im = P3 - P1 - P2 (P1 = Ar Br, P2 = Ai Bi, P3 = (Ar + Ai)(Br + Bi)) instead of
the 4 real products, J/K against the gelsy oracle.  CPU only.

  python tests/experiments/three_mult.py toy331_fr toy333_fr si_small
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


def mm3(A, B):
    """A @ B with three real products."""
    p1 = A.real @ B.real
    p2 = A.imag @ B.imag
    p3 = (A.real + A.imag) @ (B.real + B.imag)
    return (p1 - p2) + 1j * (p3 - p1 - p2)


def run(name, three):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    mesh = cell.mesh
    vol = abs(np.linalg.det(cell.a))
    N = coords.shape[0]
    Gv = R.get_Gv(cell.a, mesh)
    mm = mm3 if three else (lambda a, b: a @ b)
    ws = []
    for q, vq in enumerate(kpts):
        x4, y = o["x4"][q], o["y"][q]
        fq = np.exp(-1j * coords @ vq)
        yh = R.fft(y.T * fq, mesh)
        cg = R.get_coulG(cell.a, vq, mesh, Gv=Gv) * vol / N / N
        L = np.linalg.cholesky(x4)
        Li = sl.solve_triangular(L, np.eye(len(L)), lower=True)
        Zs = mm(Li, yh) * np.sqrt(cg)
        Mz = mm(Zs, Zs.conj().T)
        W = sl.solve_triangular(L.conj().T, sl.solve_triangular(L.conj().T, Mz, lower=False).conj().T,
                                lower=False).conj().T
        ws.append(W)
    w = np.asarray(ws)
    vj = R.get_j_kpts(o["xip"], w[0], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk = R.get_k_kpts(o["xip"], w, dm, phase)
    return abs(vj - o["vj"]).max(), abs(vk - o["vk"]).max()


if __name__ == "__main__":
    for name in sys.argv[1:]:
        for three in (False, True):
            ej, ek = run(name, three)
            print(f"{name} {'3M' if three else '4M'}: dJ {ej:.2e} dK {ek:.2e}", flush=True)
