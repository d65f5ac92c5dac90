"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Exact FFT-grid (FFTDF-equivalent) Coulomb / exchange matrices and 4-index ERIs,
restating PySCF ``pbc.df.fft_jk`` / ``FFTDF.get_eri`` semantics.
They are the *independent* known answers that pin ``oracle/isdf_ref.py``:
the reference compares ISDF J/K against FFTDF J/K (fftisdf.py:441-473) and ISDF
ERIs against ``FFTDF.get_eri`` (fftdf-with-k-lstsq.py:213-258, fails > 1e-4).
Only tests may import this module.
"""
from __future__ import annotations

import numpy as np

from .isdf_ref import fft, ifft, get_coulG, get_Gv


def exact_j(chi, dms, a, mesh):
    """[pyscf] fft_jk.get_j_kpts: chi (nk, ngrid, nao), dms (nset, nk, nao, nao)."""
    nk, ngrid, nao = chi.shape
    vol = abs(np.linalg.det(a))
    coulG = get_coulG(a, np.zeros(3), mesh)
    out = []
    for dm in dms:
        rho = np.einsum("kgm,kmn,kgn->g", chi, dm, chi.conj()) / nk
        v = ifft((coulG * fft(rho[None], mesh)[0])[None], mesh)[0]
        out.append(np.einsum("kgm,g,kgn->kmn", chi.conj(), v, chi) * (vol / ngrid))
    return np.asarray(out)


def exact_k(chi, dms, a, mesh, kpts, coords):
    """[pyscf] fft_jk.get_k_kpts (exxdiv=None): pair chi*_{k1,m} chi_{k2,l}, q = k2-k1,
    demodulated by exp(-i q.r), weight (vol/ngrid)/nk."""
    nk, ngrid, nao = chi.shape
    vol = abs(np.linalg.det(a))
    Gv = get_Gv(a, mesh)
    out = np.zeros((len(dms), nk, nao, nao), complex)
    for k2 in range(nk):
        for k1 in range(nk):
            q = kpts[k2] - kpts[k1]
            coulG = get_coulG(a, q, mesh, Gv=Gv)
            em = np.exp(-1j * coords @ q)
            pair = (chi[k1].conj().T[:, None, :] * chi[k2].T[None, :, :]) * em   # (m, l, g)
            vG = fft(pair.reshape(-1, ngrid), mesh) * coulG
            vR = ifft(vG, mesh).reshape(nao, nao, ngrid) * em.conj()
            for i, dm in enumerate(dms):
                # K[m,n] += sum_{l,s,g} vR[m,l,g] D[l,s] chi*_{k2,s}(g) chi_{k1,n}(g)
                u = dm[k2] @ chi[k2].conj().T                          # (l, g)
                t = np.einsum("mlg,lg->mg", vR, u)
                out[i, k1] += t @ chi[k1] * (vol / ngrid) / nk
    return out


def exact_eri(chi, a, mesh, kpts, coords, k1, k2, k3, k4):
    """[pyscf] FFTDF.get_eri for one k-quartet; chemists' (m k1, n k2 | k k3, l k4)."""
    nk, ngrid, nao = chi.shape
    vol = abs(np.linalg.det(a))
    q = kpts[k2] - kpts[k1]
    coulG = get_coulG(a, q, mesh)
    em = np.exp(-1j * coords @ q)
    p12 = (chi[k1].conj().T[:, None, :] * chi[k2].T[None, :, :] * em).reshape(-1, ngrid)
    v = ifft(fft(p12, mesh) * coulG, mesh) * em.conj()
    p34 = (chi[k3].conj().T[:, None, :] * chi[k4].T[None, :, :]).reshape(-1, ngrid)
    eri = v @ p34.T * (vol / ngrid)
    return eri.reshape(nao, nao, nao, nao)
