"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

NumPy/SciPy restatement of the reference's k-point FFT-ISDF hot path
(``/root/reference/fftisdf.py``).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline — never as the product path.

Parity status: the reference cannot run here (PySCF, h5py, opt_einsum absent;
SURVEY.md §8c), so this restatement is pinned by known-answer tests instead
(``oracle/exact_ref.py``: ISDF J/K vs exact FFT-grid J/K, the Gamma fit KAT of
fftisdf-supercell-2.py:62-85, the reality invariants of fftisdf.py:43,81,216 and
Phi = sqrt(nk)·IDFT).  Against the reference itself: **parity unpinned**.

Every function cites the reference line range it restates.  PySCF helpers on
the path (get_phase, get_Gv, get_coulG, tools.fft/ifft, pivoted_cholesky) are
restated here independently of the product package.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg
from scipy.linalg import lapack


# ---------------------------------------------------------------------------
# PySCF helpers restated
# ---------------------------------------------------------------------------
def _cartesian_prod(arrays):
    g = np.meshgrid(*[np.asarray(a) for a in arrays], indexing="ij")
    return np.stack([x.ravel() for x in g], axis=1)


def get_kpts(a, kmesh):
    """[pyscf] Cell.get_kpts(kmesh), wrap_around=False (fftisdf.py:322)."""
    b = 2 * np.pi * np.linalg.inv(a).T
    return _cartesian_prod([np.arange(n) / n for n in kmesh]) @ b


def get_phase(a, kpts, kmesh):
    """[pyscf] k2gamma.get_phase(cell, kpts, kmesh, wrap_around=False) -> phase (fftisdf.py:28)."""
    ts = _cartesian_prod([np.arange(n) for n in kmesh]) @ a
    return np.exp(1j * ts @ np.asarray(kpts).T) / np.sqrt(len(kpts))


def get_Gv(a, mesh):
    """[pyscf] cell.get_Gv(mesh) (fftisdf.py:91)."""
    b = 2 * np.pi * np.linalg.inv(a).T
    return _cartesian_prod([np.fft.fftfreq(n, 1.0 / n) for n in mesh]) @ b


def get_coulG(a, k, mesh, Gv=None, wrap_around=True, omega=None):
    """[pyscf] tools.get_coulG(cell, k, mesh, Gv), exxdiv=None (fftisdf.py:114).

    4*pi/|k+G|^2, |k+G|^2 == 0 -> 0; for k != 0 the k+G vectors are wrapped by the
    box edge (mesh//2 + 1/2)·b and entries exactly on the edge are zeroed.
    omega (get_coulG's range separation; used by the next-4 omega path, which the reference's
    get_jk rejects): > 0 long range x exp(-|k+G|^2/4w^2); < 0 short range x (1 - exp(...)) with
    the |k+G| = 0 limit pi/w^2.
    """
    b = 2 * np.pi * np.linalg.inv(a).T
    if Gv is None:
        Gv = get_Gv(a, mesh)
    k = np.asarray(k, float)
    kG = k + Gv if abs(k).sum() > 1e-9 else Gv.copy()
    on_boundary = np.zeros(len(Gv), bool)
    if wrap_around and abs(k).sum() > 1e-9:
        box_edge = (np.asarray(mesh) // 2 + 0.5)[:, None] * b
        red = np.linalg.solve(box_edge.T, kG.T).T.round(9)
        edge = red.astype(int)
        for i in range(3):
            on_boundary |= red[:, i] == 1
            on_boundary |= red[:, i] == -1
            kG[edge[:, i] == 1] -= 2 * box_edge[i]
            kG[edge[:, i] == -1] += 2 * box_edge[i]
    g2 = np.einsum("gi,gi->g", kG, kG)
    with np.errstate(divide="ignore"):
        coulG = 4 * np.pi / g2
    coulG[g2 == 0] = 0
    if omega:
        f = np.exp(-0.25 * g2 / omega**2)
        if omega > 0:
            coulG *= f
        else:
            coulG *= 1 - f
            coulG[g2 == 0] = np.pi / omega**2
    coulG[on_boundary] = 0
    return coulG


def _fft_workers():
    """Threads for the oracle's FFTs (PySCF's tools.fft is a multithreaded FFTW/NumPy engine;
    the transform itself is the same): the process's CPU share — OMP_NUM_THREADS where the
    host sets it (the GPU pool gives each one-GPU box 16 of the host's CPUs), else the CPUs this
    process may run on."""
    import os
    n = os.environ.get("OMP_NUM_THREADS", "")
    if n.isdigit() and int(n) > 0:
        return int(n)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return os.cpu_count() or 1


def fft(f, mesh):
    """[pyscf] tools.fft: unnormalised fftn over mesh (fftisdf.py:113)."""
    import scipy.fft
    f = np.asarray(f)
    n = f.shape[0]
    return scipy.fft.fftn(f.reshape(n, *mesh), axes=(1, 2, 3),
                          workers=_fft_workers()).reshape(n, -1)


def ifft(f, mesh):
    """[pyscf] tools.ifft: ifftn (1/N) over mesh (fftisdf.py:118)."""
    import scipy.fft
    f = np.asarray(f)
    n = f.shape[0]
    return scipy.fft.ifftn(f.reshape(n, *mesh), axes=(1, 2, 3),
                           workers=_fft_workers()).reshape(n, -1)


def pivoted_cholesky(A, tol=-1.0):
    """[pyscf] lib.scipy_helper.pivoted_cholesky -> (chol, perm, rank) (fftisdf.py:381-382).

    LAPACK dpstrf (upper), 0-based permutation, rows past the rank zeroed.
    """
    n = A.shape[0]
    c, piv, rank, info = lapack.dpstrf(np.array(A, order="F", copy=True), tol=tol, lower=False)
    if info < 0:
        raise RuntimeError("Pivoted Cholesky factorization failed.")
    c = np.triu(c)
    c[rank:, :] = 0
    return c, piv - 1, rank


# ---------------------------------------------------------------------------
# fftisdf.py restated
# ---------------------------------------------------------------------------
def select_interpolation_points(x0, nao, c0):
    """fftisdf.py:357-388.  x0: (nk, ng0, nao) Bloch AOs on the parent grid.

    Returns (perm[:nip], rank, nip, x4).  The Gram x4 = (sum_q Re(x0_q* x0_q^T))^2 / nk.
    """
    nkpt, ng = x0.shape[:2]
    x2 = np.zeros((ng, ng))
    for q in range(nkpt):                               # :376-378
        x2 += (x0[q].conj() @ x0[q].T).real
    x4 = x2 * x2 / nkpt                                 # :379
    chol, perm, rank = pivoted_cholesky(x4)             # :381-382
    nip = min(int(nao * c0), rank)                      # :383
    return perm[:nip], rank, nip, x4


def select_points_svd_script(x_gamma, ng, cisdf):
    """fftdf-with-k-svd.py:49-57: Gamma-only Gram x4 = (x x^T)**2 of the parent-grid AOs
    x_gamma (ng, nao), dpstrf with tol=1e-32, nip = int(ng * cisdf) — not capped by the rank, so
    perm[:nip] runs into the part of dpstrf's permutation past its stop.  Returns
    (perm[:nip], rank, x4)."""
    x = np.asarray(x_gamma)
    x4 = (lambda v: (v @ v.T) ** 2)(x)                                 # :50
    chol, perm, rank = pivoted_cholesky(x4, tol=1e-32)                 # :53
    nip = int(ng * cisdf)                                              # :54
    return perm[:nip], rank, x4


def build_x4(xip, phase):
    """fftisdf.py:38-48: x2_k, x2_s (real), x4_s = x2_s**2, x4_k = Phi^H x4_s."""
    nkpt, nip, nao = xip.shape
    nimg = phase.shape[0]
    x2_k = np.asarray([xq.conj() @ xq.T for xq in xip])          # :38
    x2_s = (phase @ x2_k.reshape(nkpt, -1)).reshape(nimg, nip, nip)  # :41-42
    assert abs(x2_s.imag).max() < 1e-10                           # :43
    x4_s = x2_s * x2_s                                            # :45
    x4_k = phase.conj().T @ x4_s.reshape(nimg, -1)                # :46
    return x4_k.reshape(nkpt, nip, nip)


def build_y(f_k, xip, phase):
    """fftisdf.py:72-85 for one grid block: f_k (nk, blk, nao) -> y_k (nk, blk, nip)."""
    nkpt, nblk, nao = f_k.shape
    nip = xip.shape[1]
    nimg = phase.shape[0]
    fx_k = np.asarray([f.conj() @ x.T for f, x in zip(f_k, xip)])   # :76
    fx_s = (phase @ fx_k.reshape(nkpt, -1)).reshape(nimg, nblk, nip)  # :79-80
    assert abs(fx_s.imag).max() < 1e-10                              # :81
    y_s = fx_s * fx_s                                                # :83
    y_k = phase.T @ y_s.reshape(nimg, -1)                            # :84
    return y_k.reshape(nkpt, nblk, nip)


def svd_solve(x4_q, rhs, cut=np.finfo(float).eps):
    """Truncated SVD pseudo-solve z = V_r S_r^-1 U_r^H rhs, s_i > cut * s_0 (cut = machine eps,
    scipy lstsq's default rcond): what the SVD fit of fftdf-with-k-svd.py:158-164
    intends (that code keeps a fixed rank 300 and leaves z in the rotated basis, SURVEY
    Appendix B; restated here without those defects)."""
    u, sv, vh = scipy.linalg.svd(x4_q, full_matrices=False)
    r = int((sv > cut * sv[0]).sum())
    return vh[:r].conj().T @ ((u[:, :r].conj().T @ rhs) / sv[:r, None]), r


def fit_and_coulomb(x4_q, y_q, vq, coord, a, mesh, vol, Gv=None, omega=None, solver="gelsy"):
    """fftisdf.py:97-121 for one q: gelsy fit (or the SVD pseudo-solve) then FFT Coulomb ->
    (W_q, rank)."""
    ngrid = coord.shape[0]
    fq = np.exp(-1j * coord @ vq)                                     # :99
    if solver == "svd":
        z_q, rank = svd_solve(x4_q, y_q.T)                            # fftdf-with-k-svd.py:158
    else:
        res = scipy.linalg.lstsq(x4_q, y_q.T, lapack_driver="gelsy")  # :108
        z_q, rank = res[0], res[2]
    zeta = fft(z_q * fq, mesh)                                        # :113
    zeta *= get_coulG(a, vq, mesh, Gv=Gv, omega=omega)                # :114
    zeta *= vol / ngrid                                               # :115
    zeta = ifft(zeta, mesh)                                           # :118
    zeta *= fq.conj()                                                 # :119
    return zeta @ z_q.conj().T, rank                                  # :121


def build(xip, f_k, coord, a, kmesh, mesh, blksize=8000, progress=False, omega=None,
          solver="gelsy"):
    """fftisdf.py:22-128 given the interpolation-point AOs ``xip`` and the grid AOs ``f_k``.

    Returns dict(x=xip, w0=W_0, wq=W_q, ranks=[...], y=y, x4=x4_k).
    """
    kpts = get_kpts(a, kmesh)
    phase = get_phase(a, kpts, kmesh)
    nkpt, nip, nao = xip.shape
    ngrid = coord.shape[0]
    vol = abs(np.linalg.det(a))
    x4_k = build_x4(xip, phase)
    y = np.empty((nkpt, ngrid, nip), complex)
    for g0 in range(0, ngrid, blksize):                               # :72
        g1 = min(g0 + blksize, ngrid)
        y[:, g0:g1] = build_y(f_k[:, g0:g1], xip, phase)
    Gv = get_Gv(a, mesh)
    wq, ranks = [], []
    for q, vq in enumerate(kpts):                                     # :97
        w, r = fit_and_coulomb(x4_k[q], y[q], vq, coord, a, mesh, vol, Gv, omega, solver)
        wq.append(w)
        ranks.append(r)
        if progress:
            print(f"oracle fit q {q + 1}/{nkpt} rank {r}", flush=True)
    wq = np.asarray(wq).reshape(nkpt, nip, nip)                       # :124
    return dict(x=xip, w0=wq[0], wq=wq, ranks=ranks, x4=x4_k, y=y)


def get_j_kpts(xk, w0, dms, kpts_band_is_zero=False, xband=None):
    """fftisdf.py:133-171.  dms: (nset, nk, nao, nao).  xband (nband, nip, nao): the AOs at the
    interpolation points for band k-points (kpts_band, which the reference asserts away at
    :164): J there from the same v."""
    nset, nkpt, nao = dms.shape[:3]
    rho = np.einsum("kIm,kIn,xkmn->xI", xk, xk.conj(), dms, optimize=True) / nkpt  # :155-156
    v = np.einsum("IJ,xJ->xI", w0, rho, optimize=True)                            # :159
    xo = xk if xband is None else xband
    vj = np.einsum("kIm,kIn,xI->xkmn", xo.conj(), xo, v, optimize=True)           # :166
    if kpts_band_is_zero:                                                         # :169-170
        vj = vj.real
    return vj


def get_k_kpts(xk, wq, dms, phase):
    """fftisdf.py:173-228.  dms: (nset, nk, nao, nao)."""
    nkpt, nip, nao = xk.shape
    nimg = phase.shape[0]
    ws = (phase @ wq.reshape(nkpt, -1)).reshape(nimg, nip, nip)      # :205-206
    ws = ws.real * np.sqrt(nkpt)                                      # :207
    out = []
    for dm in dms:                                                    # :210
        rhok = np.asarray([x @ d @ x.conj().T for x, d in zip(xk, dm)]) / nkpt  # :211-212
        rhos = phase @ rhok.reshape(nkpt, -1)                         # :215
        assert abs(rhos.imag).max() < 1e-10                           # :216
        rhos = rhos.real.reshape(nimg, nip, nip)                      # :217
        vs = ws * rhos.transpose(0, 2, 1)                             # :219
        vk = (phase.T @ vs.reshape(nimg, -1)).reshape(nkpt, nip, nip)  # :222-223
        out.append([x.conj().T @ v @ x for x, v in zip(xk, vk)])      # :225
    return np.asarray(out).reshape(len(dms), nkpt, nao, nao)
