"""How well-posed is parity with gelsy when x4_q is rank-deficient (nip above the numerical
rank: the toy cases and the reference demo's c0 = 40, fftisdf.py:461)?  CPU only.

  python tests/experiments/gelsy_sensitivity.py toy331 [toy222 ...]

For each case, J/K from the fit variants below are compared with gelsy at rcond = eps (the
oracle, fftisdf.py:108) and with the exact FFT-grid J/K:

  gelsy(rc)    scipy lstsq gelsy at other rcond values (gelsy's own sensitivity)
  qrcp-basic   geqp3 (gelsy's QRCP) + rank cut |R_ii| > rc |R_00| + basic solution
  qrcp-rz      geqp3 + the complete-orthogonal (RZ) step: the minimum-norm solution of the
               truncated problem, i.e. gelsy's algorithm with a plain rank cut instead of its
               incremental condition estimator
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE)]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402

from cases import inputs, oracle  # noqa: E402
from oracle import isdf_ref as R, exact_ref as E  # noqa: E402

EPS = np.finfo(float).eps


def z_gelsy(x4, y, rc):
    z, _, r, _ = sl.lstsq(x4, y, lapack_driver="gelsy", cond=rc)
    return z, r


def qrcp(x4, rc):
    Q, Rm, P = sl.qr(x4, pivoting=True)
    d = abs(np.diag(Rm))
    r = int((d > rc * d[0]).sum())
    return Q, Rm, P, r


def z_qrcp_basic(x4, y, rc):
    Q, Rm, P, r = qrcp(x4, rc)
    c = Q[:, :r].conj().T @ y
    z = np.zeros((x4.shape[1], y.shape[1]), complex)
    z[P[:r]] = sl.solve_triangular(Rm[:r, :r], c)
    return z, r


def z_qrcp_rz(x4, y, rc):
    Q, Rm, P, r = qrcp(x4, rc)
    c = Q[:, :r].conj().T @ y
    # [R11 R12] = T Z (RZ): QR of [R11 R12]^H = Zq Tq, so [R11 R12] = Tq^H Zq^H
    Zq, Tq = sl.qr(Rm[:r].conj().T, mode="economic")
    w = sl.solve_triangular(Tq.conj().T, c, lower=True)
    zp = Zq @ w
    z = np.zeros((x4.shape[1], y.shape[1]), complex)
    z[P] = zp
    return z, r


def w_from_z(z, vq, coords, cell, mesh):
    vol = abs(np.linalg.det(cell.a))
    N = coords.shape[0]
    fq = np.exp(-1j * coords @ vq)
    zeta = R.fft(z * fq, mesh) * R.get_coulG(cell.a, vq, mesh) * vol / N
    zeta = R.ifft(zeta, mesh) * fq.conj()
    return zeta @ z.conj().T


def run(name):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    ex_j = E.exact_j(chi, dm, cell.a, cell.mesh)
    ex_k = E.exact_k(chi, dm, cell.a, cell.mesh, kpts, coords)
    print(f"{name}: nip {o['nip']} gelsy ranks {o['ranks']}; gelsy vs exact dJ "
          f"{abs(o['vj'] - ex_j).max():.2e} dK {abs(o['vk'] - ex_k).max():.2e}", flush=True)
    variants = [("gelsy", z_gelsy, 2 * EPS), ("gelsy", z_gelsy, 4 * EPS), ("gelsy", z_gelsy, 1e-15),
                ("gelsy", z_gelsy, 0.5 * EPS),
                ("qrcp-basic", z_qrcp_basic, EPS), ("qrcp-rz", z_qrcp_rz, EPS),
                ("qrcp-rz", z_qrcp_rz, 4 * EPS)]
    for vname, fn, rc in variants:
        ws, rs = [], []
        for q, vq in enumerate(kpts):
            z, r = fn(o["x4"][q], o["y"][q].T, rc)
            ws.append(w_from_z(z, vq, coords, cell, cell.mesh))
            rs.append(r)
        w = np.asarray(ws)
        vj = R.get_j_kpts(o["xip"], w[0], dm, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
        vk = R.get_k_kpts(o["xip"], w, dm, phase)
        print(f"  {vname:10s} rc {rc:.1e} ranks {min(rs)}-{max(rs)}: vs gelsy dJ "
              f"{abs(vj - o['vj']).max():.2e} dK {abs(vk - o['vk']).max():.2e} | vs exact dJ "
              f"{abs(vj - ex_j).max():.2e} dK {abs(vk - ex_k).max():.2e}", flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["toy331", "toy222"]:
        run(n)
