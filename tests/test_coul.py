"""next-3: the reference scripts' ``get_coul`` surface and ERI check loop.

CPU tests: the host logic (``cutoff_to_mesh``, k-conservation tables, the FFTDF holder).
GPU tests: ``get_coul`` / ``get_coul_pinv`` through the HIP path against the oracle on the
GPU-chosen point set, and ``check_eri`` (fftdf-with-k-lstsq.py:208-258) against exact ERIs.
"""
import numpy as np
import pytest

from fisdf import coul
from fisdf.cell import cartesian_prod


def test_cutoff_to_mesh_cubic():
    """Cubic cell: |b_i| = 2 pi / L, so mesh_i = ceil(2 sqrt(2 ke) L / (2 pi))."""
    L = 6.0
    for ke in (5.0, 20.0, 100.0):
        m = coul.cutoff_to_mesh(np.eye(3) * L, ke)
        assert (m == int(np.ceil(np.sqrt(2 * ke) * L / np.pi))).all()
    # monotone in the cutoff, one entry per axis, on a non-orthogonal cell
    a = (np.ones((3, 3)) - np.eye(3)) * 3.5668 / 0.52917721092
    m1, m2 = coul.cutoff_to_mesh(a, 10.0), coul.cutoff_to_mesh(a, 20.0)
    assert m1.shape == (3,) and (m2 >= m1).all() and (m1 == m1[0]).all()


def test_madelung_kat():
    """tools.pbc.madelung restated: simple-cubic Madelung constant 2.8372974794806 / L for the
    Born-von Karman supercell, invariant under the Ewald splitting; scales as 1/N for an NxNxN
    k-mesh of a cubic cell."""
    from fisdf import toy_cell
    from fisdf.cell import madelung
    cell = toy_cell()
    for L in (1.0, 4.5):
        cell.a = np.eye(3) * L
        assert abs(madelung(cell, (1, 1, 1)) * L - 2.8372974794806) < 1e-12
        assert abs(madelung(cell, (3, 3, 3)) * 3 * L - 2.8372974794806) < 1e-12
    # a non-cubic cell: precision change leaves it unchanged
    cell = toy_cell()
    m1, m2 = madelung(cell, (2, 2, 1), 1e-16), madelung(cell, (2, 2, 1), 1e-12)
    assert abs(m1 - m2) < 1e-10 and m1 > 0


@pytest.mark.parametrize("kmesh", [(2, 2, 2), (3, 3, 1), (1, 1, 1), (4, 2, 3)])
def test_kconserv_tables(kmesh):
    """k1 - k2 + k3 - k4 in the reciprocal lattice; q = k2 - k1 (brute force on scaled k)."""
    from fisdf import toy_cell
    cell = toy_cell()
    kpts = cell.get_kpts(kmesh)
    k3 = coul.get_kconserv(cell, kpts, kmesh)
    k2 = coul.get_kconserv_ria(cell, kpts, kmesh)
    nk = len(kpts)
    assert k3.shape == (nk, nk, nk) and k2.shape == (nk, nk)
    a = cell.lattice_vectors()
    for i in range(nk):
        for j in range(nk):
            d = (kpts[j] - kpts[i] - kpts[k2[i, j]]) @ a.T / (2 * np.pi)
            assert abs(d - np.rint(d)).max() < 1e-9
            for k in range(nk):
                d = (kpts[i] - kpts[j] + kpts[k] - kpts[k3[i, j, k]]) @ a.T / (2 * np.pi)
                assert abs(d - np.rint(d)).max() < 1e-9
    # each row of kconserv_ria is a permutation (q runs over the whole mesh)
    assert all(sorted(k2[i]) == list(range(nk)) for i in range(nk))


def test_fftdf_holder():
    from fisdf import toy_cell
    cell = toy_cell(mesh=(10, 10, 10))
    df = coul.FFTDF(cell)
    assert df.mesh == (10, 10, 10) and df.grids.coords.shape == (1000, 3)
    with pytest.raises(NotImplementedError):
        df.get_eri(kpts=np.zeros((4, 3)))
    with pytest.raises(RuntimeError):
        coul.check_eri(df, (1, 1, 1))             # get_coul not run yet
    called = []
    df2 = coul.FFTDF(cell, eri_ref=lambda k: called.append(k.shape) or np.zeros(1))
    df2.get_eri(kpts=np.zeros((4, 3)))
    assert called == [(4, 3)]


# ---------------------------------------------------------------------------- GPU
def _toy(name):
    from cases import inputs
    return inputs(name)


def _eri_ref(cell, kmesh, chi, coords):
    from oracle import exact_ref as E
    kpts = cell.get_kpts(kmesh)

    def f(kq):
        idx = [int(np.argmin(abs(kpts - k).sum(1))) for k in kq]
        return E.exact_eri(chi, cell.lattice_vectors(), cell.mesh, kpts, coords, *idx)
    return f


@pytest.mark.gpu
def test_get_coul_pinv_vs_oracle():
    """fftdf-with-k.py get_coul: nip = min(nip, rank) points chosen on the GPU; coul_q / x_k
    against the oracle (gelsy fit) on the same point set, then J/K-level tolerance 1e-8."""
    from oracle import isdf_ref as R
    cell, kmesh, m0, c0, x0, coords, chi, dm = _toy("toy222")
    df = coul.FFTDF(cell)
    c, x = coul.get_coul_pinv(df, m0=list(m0), nip=100, kmesh=kmesh)
    nk = int(np.prod(kmesh))
    assert c.shape == (nk, 100, 100) and x.shape == (nk, 100, cell.nao_nr())
    perm = df._isdf.perm
    assert abs(x - x0[:, perm]).max() < 1e-12
    # greedy pivot order is tie-sensitive on a symmetric crystal (test_gpu_selection): the
    # first pivot is the dpstrf one, the rest is checked through the fit on the same set
    perm_ref, rank, nip, _ = R.select_interpolation_points(x0, cell.nao_nr(), 100 / cell.nao_nr())
    assert perm[0] == perm_ref[0] and len(set(perm.tolist())) == 100
    out = R.build(x0[:, perm], chi, coords, cell.a, kmesh, cell.mesh)
    err = abs(c - out["wq"]).max()
    print("coul_q vs oracle", err, "scale", abs(out["wq"]).max())
    assert err < 1e-8 * max(1.0, abs(out["wq"]).max())


@pytest.mark.gpu
def test_get_coul_lstsq_and_eri_harness():
    """fftdf-with-k-lstsq.py get_coul (tol 1e-32, nip = min(rank, 600)) and its ERI check loop
    against exact FFT-grid ERIs (fails above 1e-4 in the reference; we require 1e-6)."""
    cell, kmesh, m0, c0, x0, coords, chi, dm = _toy("toy222")
    df = coul.FFTDF(cell, eri_ref=_eri_ref(cell, kmesh, chi, coords))
    c, x = coul.get_coul(df, kmesh=kmesh, m0=list(m0))
    isdf = df._isdf
    assert isdf.nip == min(600, x0.shape[1]) or isdf.nip < 600
    assert c.shape[1] == isdf.nip and x.shape[1] == isdf.nip
    nk = int(np.prod(kmesh))
    rng = np.random.default_rng(0)
    triples = [tuple(int(t) for t in rng.integers(0, nk, 3)) for _ in range(6)] + [(0, 0, 0)]
    worst = coul.check_eri(df, kmesh, c, x, tol=1e-6, triples=triples)
    print("worst ERI error vs exact", worst)
    # the host-side einsum of the reference harness on the returned (coul_q, x_k) agrees
    k3 = coul.get_kconserv(cell, cell.get_kpts(kmesh), kmesh)
    k2 = coul.get_kconserv_ria(cell, cell.get_kpts(kmesh), kmesh)
    k1_, k2_, k3_ = triples[1]
    k4_ = k3[k1_, k2_, k3_]
    q = k2[k1_, k2_]
    ref = np.einsum("IJ,Im,In,Jk,Jl->mnkl", c[q], x[k1_].conj(), x[k2_], x[k3_].conj(), x[k4_],
                    optimize=True)
    got = isdf.get_eri(cell.get_kpts(kmesh)[[k1_, k2_, k3_, k4_]])
    assert abs(got.reshape(ref.shape) - ref).max() < 1e-10 * max(1.0, abs(ref).max())


@pytest.mark.gpu
def test_get_coul_gamma_default_kmesh():
    """kmesh=None is the reference's [1, 1, 1] (fftdf-with-k-lstsq.py:25-26): a Gamma-only
    get_coul on the C1-shaped diamond gth-szv cell; coul_q (1, nip, nip) is real-symmetric up to
    rounding and equals the oracle's W on the same points."""
    from oracle import isdf_ref as R
    cell, kmesh, m0, c0, x0, coords, chi, dm = _toy("diamond_szv_gamma")
    df = coul.FFTDF(cell)
    c, x = coul.get_coul_pinv(df, m0=list(m0), nip=int(cell.nao_nr() * c0))
    assert c.shape[0] == 1 and x.shape[0] == 1
    assert abs(c[0] - c[0].T.conj()).max() < 1e-10 * abs(c).max()
    out = R.build(x0[:, df._isdf.perm], chi, coords, cell.a, (1, 1, 1), cell.mesh)
    err = abs(c - out["wq"]).max()
    print("Gamma coul_q vs oracle", err, "scale", abs(out["wq"]).max())
    assert err < 1e-8 * max(1.0, abs(out["wq"]).max())


def test_dpstrf_permutation_tail():
    """The permutation dpstrf returns past its stop is its swap order: completing the first
    `rank` pivots by dpstrf_permutation reproduces LAPACK's whole piv (what
    fftdf-with-k-svd.py:57's perm[:nip] reads when nip exceeds the rank)."""
    from scipy.linalg import lapack
    rng = np.random.default_rng(3)
    for n, r in [(40, 7), (97, 30), (64, 64)]:
        B = rng.standard_normal((n, r))
        A = B @ B.T
        c, piv, rank, info = lapack.dpstrf(np.array(A, order="F"), tol=1e-10, lower=False)
        piv = piv - 1
        assert coul.dpstrf_permutation(piv[:rank], n).tolist() == piv.tolist(), (n, r, rank)


@pytest.mark.gpu
@pytest.mark.parametrize("nip", [36, 320])
def test_get_coul_svd_vs_oracle_and_eri_harness(nip):
    """fftdf-with-k-svd.py get_coul: Gamma-only selection Gram (x x^T)^2 with dpstrf tol=1e-32,
    nip = int(ng * cisdf), the SVD pseudo-solve.  toy222 (nao = 8 real AOs: the Gamma Gram has
    rank 36).  The GPU's pivots inside that rank are greedy-optimal to rounding (the toy crystal
    has exact ties).  nip = 36: every x4_q full rank, the solution unique — J/K against the
    oracle's SVD pseudo-solve on the same points < 1e-8 Ha.  nip = 320 (cisdf 0.44, the script's
    regime: most points past the rank, x4_q rank-deficient, the answer defined only up to the
    pseudo-solve's cut): the script's own ERI check loop against exact ERIs (its bar 1e-4), and
    J/K against the exact FFT-grid J/K no worse than the oracle's."""
    from oracle import exact_ref as E
    from oracle import isdf_ref as R
    from fisdf.cell import eval_ao_kpts
    from test_gpu_selection import residual_along
    cell, kmesh, m0, c0, x0, coords, chi, dm = _toy("toy222")
    df = coul.FFTDF(cell, eri_ref=_eri_ref(cell, kmesh, chi, coords))
    ng = int(np.prod(m0))
    cisdf = (nip + 0.5) / ng
    c, x = coul.get_coul_svd(df, kmesh=kmesh, cisdf=cisdf, m0=list(m0))
    isdf = df._isdf
    assert nip == int(ng * cisdf)
    nk = int(np.prod(kmesh))
    assert c.shape == (nk, nip, nip) and x.shape == (nk, nip, cell.nao_nr())
    perm = isdf.perm
    assert len(set(perm.tolist())) == nip and abs(x - x0[:, perm]).max() < 1e-12
    xg = eval_ao_kpts(cell, cell.gen_uniform_grids(m0), (1, 1, 1))[0].real
    perm_ref, rank_ref, x4g = R.select_points_svd_script(xg, ng, cisdf)
    sv = np.linalg.eigvalsh(x4g)[::-1]
    num_rank = int((sv > 1e-12 * sv[0]).sum())
    before, _ = residual_along(x4g, perm[:num_rank])
    tie_tol = ng * np.finfo(float).eps * np.diag(x4g).max()
    gap = max(b.max() - b[perm[j]] for j, b in enumerate(before))
    print(f"\nsvd script nip {nip}: ng {ng}, Gram numerical rank {num_rank}, GPU factorisation "
          f"stopped after {isdf.select_rank}, dpstrf after {rank_ref}; largest greedy gap over "
          f"the first {num_rank} GPU pivots {gap:.1e} (tie tolerance {tie_tol:.1e}); x4_q ranks "
          f"{np.asarray(isdf.ranks).min()}-{np.asarray(isdf.ranks).max()}")
    assert gap <= tie_tol
    out = R.build(x0[:, perm], chi, coords, cell.a, kmesh, cell.mesh, solver="svd")
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    vj0 = R.get_j_kpts(x0[:, perm], out["w0"], dm)[0]
    vk0 = R.get_k_kpts(x0[:, perm], out["wq"], dm, phase)[0]
    vj, vk = isdf.get_jk(dm[0])
    dj, dk = abs(vj - vj0).max(), abs(vk - vk0).max()
    print(f"svd script nip {nip}: GPU vs SVD oracle on the same points |dJ| {dj:.2e} |dK| {dk:.2e}")
    if nip <= num_rank:
        assert dj < 1e-8 and dk < 1e-8
        return
    vje = E.exact_j(chi, dm, cell.a, cell.mesh)[0]
    vke = E.exact_k(chi, dm, cell.a, cell.mesh, kpts, coords)[0]
    ej, ek = abs(vj - vje).max(), abs(vk - vke).max()
    ej0, ek0 = abs(vj0 - vje).max(), abs(vk0 - vke).max()
    print(f"svd script nip {nip}: vs exact FFT-grid J/K: GPU {ej:.2e} / {ek:.2e}, oracle "
          f"{ej0:.2e} / {ek0:.2e}")
    assert ej <= 1.5 * ej0 + 1e-8 and ek <= 1.5 * ek0 + 1e-8
    rng = np.random.default_rng(1)
    triples = [tuple(int(t) for t in rng.integers(0, nk, 3)) for _ in range(4)] + [(0, 0, 0)]
    worst = coul.check_eri(df, kmesh, c, x, tol=1e-4, triples=triples)
    print(f"svd script nip {nip}: worst ISDF ERI error vs exact {worst:.2e} (the script's bar 1e-4)")
