"""Full-size parity at every BASELINE configuration (C1-C5 of SURVEY.md §8d), driver-run.

Each config is built at its real size (bench.setup: same cell, basis shape, mesh, k-mesh,
nip and dm as the benchmark) by the GPU path — GPU selection, x4, y, factorisation, fit,
FFT Coulomb, W_s, get_jk — and the CPU oracle (the gelsy restatement of fftisdf.py:22-228)
then runs on the GPU's interpolation points (SURVEY.md §7 hard part (b)).  Bar: the
north_star's J/K max-abs difference < 1e-8 Ha (fftdf-with-k-lstsq.py:192-210,
fftisdf.py:432-466 compare J/K in Ha).  W_q of Gamma, a self-conjugate q and two complex q
are compared too, and the device reality monitors of fftisdf.py:43,81,216 must stay at
rounding level.  C3 costs ~140 s of oracle CPU time on the GPU box's 16 cores.
"""
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

JK_TOL = 1e-8        # Ha, north_star
M_REL_TOL = 1e-8     # max |dM_q| / max |M_q|, M_q the AO-pair projection of W_q (below)


def _gpu_build(cfg, c0=None):
    import bench
    from fisdf import ISDF
    cell, kmesh, m0, c0_cfg, x0, chi, dm = bench.setup(cfg)
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0_cfg if c0 is None else c0)
    if cfg == "c4":          # C4 is the "SVD fit" configuration (BASELINE.json configs[3])
        df.fit = "svd"
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    df.device.ctx.max_imag()                       # reset the monitors
    df.build()
    vj, vk = df.get_jk(dm)
    mi = df.device.ctx.max_imag()
    return df, cell, kmesh, x0, chi, dm, vj, vk, mi


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", ["c1", "c2", "c5", "c4", "c3"])
def test_config_parity_full_size(cfg):
    from oracle import isdf_ref as R
    df, cell, kmesh, x0, chi, dm, vj, vk, mi = _gpu_build(cfg)
    nk = int(np.prod(kmesh))
    print(f"\n{cfg}: nk {nk} nao {cell.nao_nr()} nip {df.nip} mesh {tuple(cell.mesh)} "
          f"ranks {df.ranks.min()}-{df.ranks.max()} fit {df.fit} (min-norm q {df.min_norm_slots}) "
          f"max_imag {mi}", flush=True)
    if cfg == "c4":
        assert df.min_norm_slots == len(df.fit_qs)
    # reality monitors of fftisdf.py:43 (x2_s), :81 (fx_s), :216 (rho_s), relative to O(1) data
    assert max(mi) < 1e-10, mi
    xip = x0[:, df.perm]
    coords = cell.gen_uniform_grids(cell.mesh)
    t0 = time.perf_counter()
    out = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh, progress=nk > 8)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    dms = dm[None]
    vj0 = R.get_j_kpts(xip, out["w0"], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))[0]
    vk0 = R.get_k_kpts(xip, out["wq"], dms, phase)[0]
    ej, ek = abs(vj - vj0).max(), abs(vk - vk0).max()
    print(f"{cfg}: oracle {time.perf_counter() - t0:.1f} s, gelsy ranks "
          f"{min(out['ranks'])}-{max(out['ranks'])}; |dJ| {ej:.2e} |dK| {ek:.2e} "
          f"(max|J| {abs(vj0).max():.3f}, max|K| {abs(vk0).max():.3f})", flush=True)
    assert vj.shape == dm.shape and vk.shape == dm.shape
    assert ej < JK_TOL and ek < JK_TOL
    # W_q of Gamma, one self-conjugate q (2 k_q in the reciprocal lattice) and two complex q.
    # W_q itself is as ill-conditioned as x4_q (measured rel |dW| 2.6e-3 at C5, 2.7e-6 at C3
    # between the two solvers) — the well-conditioned quantity J/K and the ERIs see is its
    # AO-pair projection M_q = B^T W_q conj(B), B[I, mn] = conj(X_0[I, m]) X_q[I, n]: the
    # (m 0, n q | l q, k 0) ERI block of fftdf-with-k-lstsq.py:221-232 (pair momentum q on
    # both sides, the only combination W_q is fitted for)
    wq = df._wq
    ks = np.stack(np.unravel_index(np.arange(nk), tuple(kmesh)), 1)
    selfc = [q for q in range(1, nk) if not ((2 * ks[q]) % kmesh).any()]
    cplxq = [q for q in range(nk) if ((2 * ks[q]) % kmesh).any()]
    check = [0] + selfc[:1] + cplxq[:1] + cplxq[len(cplxq) // 2:len(cplxq) // 2 + 1]
    for q in check:
        B = (xip[0].conj()[:, :, None] * xip[q][:, None, :]).reshape(df.nip, -1)
        m_gpu = B.T @ (wq[q] @ B.conj())
        m_ref = B.T @ (out["wq"][q] @ B.conj())
        rel = abs(m_gpu - m_ref).max() / abs(m_ref).max()
        relw = abs(wq[q] - out["wq"][q]).max() / abs(out["wq"][q]).max()
        print(f"{cfg}: q {q} rel |dM_q| {rel:.2e} (raw rel |dW_q| {relw:.2e})", flush=True)
        assert rel < M_REL_TOL, (q, rel)


def _oracle_jk(cell, kmesh, x0, chi, dm, perm):
    """The reference CPU path (fftisdf.py:22-228, gelsy fit) on the interpolation points perm."""
    from oracle import isdf_ref as R
    xip = x0[:, perm]
    out = R.build(xip, chi, cell.gen_uniform_grids(cell.mesh), cell.a, kmesh, cell.mesh)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    dms = dm[None]
    vj = R.get_j_kpts(xip, out["w0"], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))[0]
    vk = R.get_k_kpts(xip, out["wq"], dms, phase)[0]
    return vj, vk, out


SEL_RATIO = 1.5      # GPU build's error vs exact FFT-grid J/K, relative to the reference's own


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_jk_vs_reference_selection(cfg):
    """End to end against the reference path on ITS OWN selection (LAPACK dpstrf pivots,
    fftisdf.py:357-388), not on the GPU's points.

    The parent-grid Gram of the diamond cell has exactly tied diagonal entries (symmetry-
    equivalent grid points), so dpstrf's greedy pivots are decided by the last bits of x2: the
    reference itself picks a different point set when x2 is summed in another valid order (C2:
    pivots diverge at step 1, 51 % shared, J/K differ by 1.6e-3 / 2.5e-4 Ha —
    tests/experiments/selection_sensitivity.py, profiles/r03_selection_sensitivity.log).  J/K of
    two selections therefore differ at the ISDF-approximation level, not at rounding level, and
    the 1e-8 bar applies on a common point set (test_config_parity_full_size).  What is asserted
    here is that the GPU's selection is as good as the reference's: its error against the exact
    FFT-grid J (and K at C2; oracle/exact_ref.py, PySCF fft_jk semantics) is within SEL_RATIO of
    the reference build's, and the GPU-vs-reference difference is explained by that error."""
    from oracle import exact_ref as E
    from oracle import isdf_ref as R
    df, cell, kmesh, x0, chi, dm, vj, vk, mi = _gpu_build(cfg)
    t0 = time.perf_counter()
    perm_ref, rank_ref, nip_ref, _ = R.select_interpolation_points(x0, cell.nao_nr(), df.c0)
    shared = len(set(perm_ref.tolist()) & set(df.perm.tolist())) / len(perm_ref)
    first = next((i for i in range(min(len(perm_ref), len(df.perm)))
                  if perm_ref[i] != df.perm[i]), None)
    vj_ref, vk_ref, _ = _oracle_jk(cell, kmesh, x0, chi, dm, perm_ref)
    dj, dk = abs(vj - vj_ref).max(), abs(vk - vk_ref).max()
    print(f"\n{cfg}: GPU vs reference on its own dpstrf pivots (nip {nip_ref}, first divergence "
          f"{first}, shared {100 * shared:.0f}%): |dJ| {dj:.2e} |dK| {dk:.2e} "
          f"(oracle {time.perf_counter() - t0:.1f} s)", flush=True)
    if np.array_equal(perm_ref, df.perm):
        assert dj < JK_TOL and dk < JK_TOL
        return
    t0 = time.perf_counter()
    kpts = R.get_kpts(cell.a, kmesh)
    dms = dm[None]
    vje = E.exact_j(chi, dms, cell.a, cell.mesh)[0]
    if abs(kpts).max() < 1e-9:
        vje = vje.real
    ej_gpu, ej_ref = abs(vj - vje).max(), abs(vj_ref - vje).max()
    msg = f"{cfg}: vs exact FFT-grid J: GPU {ej_gpu:.2e}, reference {ej_ref:.2e}"
    if cfg == "c2":   # exact K: nk^2 pair FFTs, affordable at 2x2x2
        vke = E.exact_k(chi, dms, cell.a, cell.mesh, kpts, cell.gen_uniform_grids(cell.mesh))[0]
        ek_gpu, ek_ref = abs(vk - vke).max(), abs(vk_ref - vke).max()
        msg += f"; K: GPU {ek_gpu:.2e}, reference {ek_ref:.2e}"
        assert ek_gpu <= SEL_RATIO * ek_ref, msg
        assert dk <= 2 * max(ek_gpu, ek_ref), msg
    print(msg + f" (exact {time.perf_counter() - t0:.1f} s)", flush=True)
    assert ej_gpu <= SEL_RATIO * ej_ref, msg
    assert dj <= 2 * max(ej_gpu, ej_ref), msg


def _gelsy_jk(cell, kmesh, x0, chi, dm, perm, cond):
    """J/K of the reference path with gelsy at rcond `cond` (None: scipy's default, eps)."""
    import scipy.linalg as sl
    from oracle import isdf_ref as R
    xip = x0[:, perm]
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    coords = cell.gen_uniform_grids(cell.mesh)
    x4 = R.build_x4(xip, phase)
    N = coords.shape[0]
    yall = np.empty((len(kpts), N, xip.shape[1]), complex)
    for g0 in range(0, N, 8000):
        yall[:, g0:g0 + 8000] = R.build_y(chi[:, g0:g0 + 8000], xip, phase)
    Gv = R.get_Gv(cell.a, cell.mesh)
    ws, ranks = [], []
    for q, vq in enumerate(kpts):
        fq = np.exp(-1j * coords @ vq)
        z, _, r, _ = sl.lstsq(x4[q], yall[q].T, cond=cond, lapack_driver="gelsy")  # :108
        zeta = R.fft(z * fq, cell.mesh) * R.get_coulG(cell.a, vq, cell.mesh, Gv=Gv) * (cell.vol / N)
        ws.append((R.ifft(zeta, cell.mesh) * fq.conj()) @ z.conj().T)
        ranks.append(r)
    w = np.asarray(ws)
    dms = dm[None]
    return (R.get_j_kpts(xip, w[0], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))[0],
            R.get_k_kpts(xip, w, dms, phase)[0], ranks)


@pytest.mark.timeout(900)
def test_min_norm_fit_full_size_rank_regime():
    """The reference demo's regime at full size (fftisdf.py:455-461: c0 = 40, nip reaches the
    parent-Gram rank through :383): C2's cell, basis, mesh and k-mesh with c0 large enough that
    nip = rank (~1500-1600 points), so every x4_q is rank-deficient (cond ~1e16: directions at
    the rounding level decide the solution) and the fit takes the minimum-norm path (DESIGN
    §3.4).  Here the reference's own answer is only defined to the level its solver moves under
    a change of rcond: gelsy at 4x and 1/4x its default rcond differs from itself by ~1.5e-7 Ha
    (J) / ~2.5e-8 (K) (tests/experiments/rank_regime_c2.py, profiles/r03_rank_regime_c2.log),
    above the 1e-8 bar.  The fit's rank cut (fit_tol 4.2e-15) is the one whose ranks follow
    gelsy's here (tests/experiments/rank_rule_c2.py).  Asserted: the GPU's J/K sit inside that band
    around gelsy at its default rcond (1x; round 4's 1e-14 cut needed 1.4x), on the GPU's points;
    the measured |dJ| / |dK| are printed against the 1e-8 bar, which no solver other than gelsy
    itself meets in this regime."""
    df, cell, kmesh, x0, chi, dm, vj, vk, mi = _gpu_build("c2", c0=1e4)
    ng0 = x0.shape[1]
    print(f"\nc2 rank regime: nip {df.nip} (parent grid {ng0}), x4_q ranks "
          f"{df.ranks.min()}-{df.ranks.max()}, min-norm q {df.min_norm_slots}/{len(df.fit_qs)} "
          f"max_imag {mi}", flush=True)
    assert df.nip < ng0 and df.min_norm_slots == len(df.fit_qs)
    assert max(mi) < 1e-10, mi
    t0 = time.perf_counter()
    eps = np.finfo(float).eps
    vj0, vk0, r0 = _gelsy_jk(cell, kmesh, x0, chi, dm, df.perm, None)
    band_j = band_k = 0.0
    for cond in (4 * eps, eps / 4):
        vj1, vk1, r1 = _gelsy_jk(cell, kmesh, x0, chi, dm, df.perm, cond)
        band_j = max(band_j, abs(vj1 - vj0).max())
        band_k = max(band_k, abs(vk1 - vk0).max())
        print(f"c2 rank regime: gelsy rcond {cond:.1e} (ranks {min(r1)}-{max(r1)}) vs default "
              f"(ranks {min(r0)}-{max(r0)}): |dJ| {abs(vj1 - vj0).max():.2e} "
              f"|dK| {abs(vk1 - vk0).max():.2e}", flush=True)
    ej, ek = abs(vj - vj0).max(), abs(vk - vk0).max()
    print(f"c2 rank regime: GPU vs gelsy: |dJ| {ej:.2e} |dK| {ek:.2e} (bar 1e-8); gelsy's own "
          f"rcond band |dJ| {band_j:.2e} |dK| {band_k:.2e} (GPU at {ej / band_j:.2f} / "
          f"{ek / band_k:.2f} of the band; oracle {time.perf_counter() - t0:.1f} s)", flush=True)
    assert ej <= band_j and ek <= band_k


# C2 / C3 with the second C moved off its symmetric site (Angstrom): no symmetry maps the parent
# grid onto itself, so the parent-grid Gram has no exactly tied diagonal entries
# (this shift's smallest gap between the two largest residual diagonals along dpstrf's order,
# relative to max diag: C2 3.7e-9, C3 2.3e-11, against rounding at ~1e-13)
DISPLACED = {"c2d": ("c2", (0.11, -0.023, 0.067)), "c3d": ("c3", (0.11, -0.023, 0.067))}


def _displaced_inputs(name):
    import bench
    from fisdf import cell as C
    cfg, shift = DISPLACED[name]
    kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS[cfg]
    cell = C.diamond_cell(basis=basis, mesh=mesh, shift=shift)
    nao = cell.nao_nr()
    c0 = (nip + 0.5) / nao
    x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
    chi = C.eval_ao_kpts(cell, cell.gen_uniform_grids(mesh), kmesh)
    dm = C.make_dm(nao, kmesh, cell, seed=1234)
    return cell, kmesh, m0, c0, x0, chi, dm


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c2d", "c3d"])
def test_end_to_end_own_selection(name):
    """North star without injected points (VERDICT r03 ask 3): the GPU build with ITS OWN
    selection against the reference's whole CPU path with ITS OWN selection (LAPACK dpstrf,
    fftisdf.py:357-388, then :22-228 with gelsy) on a cell without exact pivot ties.  Asserted:
    identical pivots, then |dJ|, |dK| < 1e-8 Ha.  Should the greedy orders part anyway, the
    residual-diagonal gap at the first divergence is printed and must be a rounding-level tie
    (test_gpu_selection.py's certificate); J/K are then compared on the GPU's points."""
    from fisdf import ISDF
    from oracle import isdf_ref as R
    from test_gpu_selection import residual_along
    cell, kmesh, m0, c0, x0, chi, dm = _displaced_inputs(name)
    nao = cell.nao_nr()
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    df.build()
    vj, vk = df.get_jk(dm)
    t0 = time.perf_counter()
    perm_ref, rank_ref, nip_ref, x4 = R.select_interpolation_points(x0, nao, c0)
    assert len(df.perm) == nip_ref
    same = df.perm == perm_ref
    first = int(np.argmin(same)) if not same.all() else nip_ref
    msg = f"\n{name}: nip {nip_ref}, GPU and dpstrf pivots identical for {first}/{nip_ref} steps"
    perm_jk = perm_ref
    if first < nip_ref:
        tie_tol = x4.shape[0] * np.finfo(float).eps * np.diag(x4).max()
        before, _ = residual_along(x4, df.perm)
        dp = before[first]
        gap = dp.max() - dp[df.perm[first]]
        msg += f"; first divergence: residual gap {gap:.2e} (tie tolerance {tie_tol:.2e})"
        print(msg, flush=True)
        assert gap <= tie_tol, msg
        perm_jk = df.perm
    vj0, vk0, _ = _oracle_jk(cell, kmesh, x0, chi, dm, perm_jk)
    dj, dk = abs(vj - vj0).max(), abs(vk - vk0).max()
    print(f"{msg}; GPU vs reference path end to end: |dJ| {dj:.2e} |dK| {dk:.2e} Ha "
          f"(max|J| {abs(vj0).max():.3f}, max|K| {abs(vk0).max():.3f}; oracle "
          f"{time.perf_counter() - t0:.1f} s)", flush=True)
    assert dj < JK_TOL and dk < JK_TOL
