"""GPU parity tests of the individual HIP engines against NumPy/SciPy (fp64 references).

Every call goes through the C-ABI (libfisdf.so) — the same symbols include/fisdf.h
declares.  Tolerances are stated per test (fp64 rounding of the op, not a model error).
"""
import ctypes as C

import numpy as np
import pytest
import scipy.linalg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    from fisdf import _lib
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    ctx = _lib.Context(0, torch.cuda.current_stream().cuda_stream)
    return torch, _lib, ctx


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def rnd(rng, *shape):
    return rng.standard_normal(shape) + 1j * rng.standard_normal(shape)


def opmat(a, op):
    if op & 1:
        a = a.swapaxes(-1, -2)
    if op & 2:
        a = a.conj()
    return a


@pytest.mark.parametrize("opA", [0, 1, 2, 3])
@pytest.mark.parametrize("opB", [0, 1, 2, 3])
def test_zgemm_ops(env, opA, opB):
    torch, L, ctx = env
    rng = np.random.default_rng(opA * 4 + opB)
    M, N, K, batch = 70, 45, 37, 3
    A = rnd(rng, batch, *((K, M) if opA & 1 else (M, K)))
    B = rnd(rng, batch, *((N, K) if opB & 1 else (K, N)))
    Cm = rnd(rng, batch, M, N)
    alpha = np.array([0.7, -0.3])
    beta = np.array([0.2, 0.5])
    ref = (alpha[0] + 1j * alpha[1]) * opmat(A, opA) @ opmat(B, opB) + (beta[0] + 1j * beta[1]) * Cm
    dA, dB, dC = dev(torch, A), dev(torch, B), dev(torch, Cm)
    ctx.call("fisdf_zgemm", opA, opB, M, N, K, alpha.ctypes.data_as(L._dp), L.ptr(dA),
             A.shape[-1], A.shape[-1] * A.shape[-2], L.ptr(dB), B.shape[-1],
             B.shape[-1] * B.shape[-2], beta.ctypes.data_as(L._dp), L.ptr(dC), N, M * N, batch, 1)
    out = dC.cpu().numpy()
    # fp64: |err| <= ~K * eps * |a||b|
    assert abs(out - ref).max() < 1e-12 * K


@pytest.mark.parametrize("M,N,K,ks", [(1, 1, 1, 1), (64, 64, 16, 1), (129, 65, 17, 1),
                                      (200, 200, 5000, 8), (600, 1, 600, 1),
                                      # edge tiles with <= 32 valid rows / columns (the waves
                                      # split by 16-blocks there)
                                      (24, 300, 50, 1), (88, 40, 33, 1), (40, 130, 70, 2),
                                      (600, 600, 300, 3)])
def test_zgemm_shapes_splitk(env, M, N, K, ks):
    torch, L, ctx = env
    rng = np.random.default_rng(M + N + K)
    A, B = rnd(rng, M, K), rnd(rng, K, N)
    dA, dB = dev(torch, A), dev(torch, B)
    dC = torch.zeros((M, N), dtype=torch.complex128, device="cuda")
    one, zero = np.array([1.0, 0.0]), np.array([0.0, 0.0])
    ctx.call("fisdf_zgemm", 0, 0, M, N, K, one.ctypes.data_as(L._dp), L.ptr(dA), K, 0, L.ptr(dB),
             N, 0, zero.ctypes.data_as(L._dp), L.ptr(dC), N, 0, 1, ks)
    ref = A @ B
    assert abs(dC.cpu().numpy() - ref).max() < 1e-12 * max(K, 16)


@pytest.mark.parametrize("n,K,ks", [(1, 7, 1), (16, 40, 1), (24, 37, 1), (40, 100, 2),
                                    (64, 64, 1), (88, 300, 4), (100, 33, 1), (600, 700, 3),
                                    # the 64 x 128 split-K kernel (n >= 128, K % 8 == 0, ks > 1):
                                    # partial tile rows / panels, dead waves above the diagonal
                                    (128, 64, 2), (130, 96, 2), (200, 256, 5), (333, 1000, 4),
                                    (600, 704, 3), (640, 1024, 8)])
def test_herk_shapes(env, n, K, ks):
    """C = A A^H through the lower-tile HERK (diagonal tiles split 3+3+2+2 over the waves,
    edge tiles by 16-blocks; the wide split-K kernel where it applies), compared with NumPy on
    the full matrix (both triangles)."""
    torch, L, ctx = env
    rng = np.random.default_rng(n * 1000 + K)
    A = rnd(rng, n, K)
    dA = dev(torch, A)
    dC = torch.full((n, n), complex(7.0, 7.0), dtype=torch.complex128, device="cuda")
    ctx.call("fisdf_herk", n, K, 1.0, L.ptr(dA), K, L.ptr(dC), n, ks)
    ref = A @ A.conj().T
    assert abs(dC.cpu().numpy() - ref).max() < 1e-12 * max(K, 16)


@pytest.mark.parametrize("mesh", [(8, 8, 8), (12, 12, 12), (13, 13, 13), (15, 15, 15),
                                  (30, 30, 30), (32, 32, 32), (36, 36, 36), (6, 10, 14)])
def test_fft3d(env, mesh):
    torch, L, ctx = env
    rng = np.random.default_rng(sum(mesh))
    rows = 5
    x = rnd(rng, rows, int(np.prod(mesh)))
    dx = dev(torch, x)
    dy = torch.empty_like(dx)
    m, mp = L.iarr(mesh)
    ctx.call("fisdf_fft3d", L.ptr(dx), L.ptr(dy), rows, mp)
    ref = np.fft.fftn(x.reshape(rows, *mesh), axes=(1, 2, 3)).reshape(rows, -1)
    err = abs(dy.cpu().numpy() - ref).max() / abs(ref).max()
    assert err < 1e-14


def _prefix_planes(n0, m0):
    """Restates half_prefix_planes (linalg.hip): planes i0 with i0 <= their partner -i0 - m0."""
    return max(i0 for i0 in range(n0) if i0 <= (-i0 - m0) % n0) + 1


@pytest.mark.parametrize("mesh", [(8, 8, 8), (12, 12, 12), (15, 15, 15), (36, 36, 36)])
@pytest.mark.parametrize("m", [(0, 0, 0), (1, 1, 1), (1, 0, 1), (0, 1, 0)])
def test_fft3d_paired(env, mesh, m):
    """The self-conjugate q's transform (fisdf_fft3d_paired: Hermitian half of the plane pass,
    the partner lines rebuilt in the axis-0 pass, real input rows) equals numpy's fftn of the
    phased real input on the prefix planes the half-grid fit reads, for both parities of m and an
    odd mesh."""
    torch, L, ctx = env
    rng = np.random.default_rng(sum(mesh) + 7 * sum(m))
    rows = 3
    y = rng.standard_normal((rows, int(np.prod(mesh))))
    kd = np.pi * np.array(m, dtype=float)
    f = [np.fft.fftfreq(n) for n in mesh]
    ph = np.exp(-1j * (f[0][:, None, None] * kd[0] + f[1][None, :, None] * kd[1]
                       + f[2][None, None, :] * kd[2]))
    ref = np.fft.fftn(y.reshape(rows, *mesh) * ph, axes=(1, 2, 3)).reshape(rows, -1)
    ncol = _prefix_planes(mesh[0], m[0]) * mesh[1] * mesh[2]
    ma, mp = L.iarr(mesh)  # the arrays stay alive as long as their pointers
    ka, kp = L.darr(kd)
    ha, hp = L.iarr(m)
    for in_real in (0, 1):
        dx = (torch.from_numpy(y).to("cuda") if in_real
              else dev(torch, y.astype(np.complex128)))
        dy = torch.full((rows, int(np.prod(mesh))), complex(7.0, 7.0), dtype=torch.complex128,
                        device="cuda")
        ctx.call("fisdf_fft3d_paired", L.ptr(dx), L.ptr(dy), rows, mp, kp, hp, in_real)
        out = dy.cpu().numpy()
        err = abs(out[:, :ncol] - ref[:, :ncol]).max() / abs(ref).max()
        assert err < 1e-14, (in_real, err)


def test_coulg(env):
    torch, L, ctx = env
    from fisdf.cell import diamond_cell, make_kpts
    from oracle import isdf_ref as R
    cell = diamond_cell(mesh=(12, 12, 12))
    kpts = make_kpts(cell, (3, 3, 3))
    m, mp = L.iarr(cell.mesh)
    a, ap = L.darr(cell.a.ravel())
    for k in kpts[[0, 1, 5, 13, 26]]:
        kk, kp = L.darr(k)
        w = torch.empty(int(np.prod(cell.mesh)), dtype=torch.float64, device="cuda")
        ctx.call("fisdf_coulg", mp, ap, kp, 1.0, 0, L.ptr(w))
        ref = R.get_coulG(cell.a, k, cell.mesh)
        np.testing.assert_allclose(w.cpu().numpy(), ref, rtol=1e-13, atol=1e-14)


def test_pivoted_cholesky_matches_dpstrf(env):
    torch, L, ctx = env
    from oracle import isdf_ref as R
    rng = np.random.default_rng(5)
    n, rk = 120, 70
    B = rng.standard_normal((n, rk)) * np.exp(-0.1 * np.arange(rk))
    A = B @ B.T
    chol, perm, rank = R.pivoted_cholesky(A)
    dA = dev(torch, A.astype(np.complex128))
    piv = np.zeros(n, np.int32)
    rnk = np.zeros(1, np.int32)
    ctx.call("fisdf_pivoted_cholesky", L.ptr(dA), n, 1, n, -1.0, piv.ctypes.data_as(L._ip),
             rnk.ctypes.data_as(L._ip))
    assert abs(int(rnk[0]) - rank) <= 1
    r = min(int(rnk[0]), rank)
    # greedy pivot order agrees with LAPACK's blocked dpstrf on a tie-free matrix
    assert np.array_equal(piv[:r - 2], perm[:r - 2])


def test_pivoted_cholesky_batched_hermitian(env):
    torch, L, ctx = env
    rng = np.random.default_rng(7)
    n, batch = 50, 4
    B = rnd(rng, batch, n, 30)
    A = B @ B.conj().swapaxes(-1, -2)
    dA = dev(torch, A)
    piv = np.zeros((batch, n), np.int32)
    rnk = np.zeros(batch, np.int32)
    ctx.call("fisdf_pivoted_cholesky", L.ptr(dA), n, batch, n, 1e-12,
             piv.ctypes.data_as(L._ip), rnk.ctypes.data_as(L._ip))
    assert (rnk == 30).all()
    for b in range(batch):
        p = piv[b, :30]
        # chosen block is well conditioned and spans A: residual of the Nystrom form ~0
        App = A[b][np.ix_(p, p)]
        Ap = A[b][:, p]
        resid = A[b] - Ap @ np.linalg.solve(App, Ap.conj().T)
        assert abs(resid).max() < 1e-8 * abs(A[b]).max()


@pytest.mark.parametrize("real", [False, True])
def test_min_norm_operator(env, real):
    """fisdf_min_norm_operator (the fit's minimum-norm path) on a rank-deficient Hermitian PSD
    matrix with a decaying spectrum: P L = Q R with Q orthonormal and Q R equal to the host's
    truncated factor of the same pivots to its conditioning, M = R^{-1} Q^H, and the solve
    z = P M^H M P^T b of a right-hand side b = x4 v in the range reproduces b (residual) with
    |z| <= |v| (minimum norm)."""
    torch, L, ctx = env
    rng = np.random.default_rng(11)
    n, rk = 150, 90
    B = rnd(rng, n, rk) if not real else rng.standard_normal((n, rk)).astype(np.complex128)
    B = B * np.exp(-0.25 * np.arange(rk))
    A = B @ B.conj().T
    dA = dev(torch, A)
    dM, dQ, dR = (torch.zeros(n, n, dtype=torch.complex128, device=dA.device) for _ in range(3))
    piv = np.zeros(n, np.int32)
    rnk = np.zeros(1, np.int32)
    ctx.call("fisdf_min_norm_operator", L.ptr(dA), n, 1e-14, L.ptr(dM), L.ptr(dQ), L.ptr(dR),
             piv.ctypes.data_as(L._ip), rnk.ctypes.data_as(L._ip))
    r = int(rnk[0])
    assert 0 < r < n and sorted(piv) == list(range(n))
    M = dM.cpu().numpy()[:r]
    Q = dQ.cpu().numpy().reshape(-1)[:n * r].reshape(n, r)
    Ri = dR.cpu().numpy().reshape(-1)[:r * r].reshape(r, r)
    Ap = A[np.ix_(piv, piv)]
    L11 = np.linalg.cholesky(Ap[:r, :r])
    Af = np.concatenate([L11, np.linalg.solve(L11, Ap[:r, r:]).conj().T])
    X = Q @ np.linalg.inv(Ri)                          # the device's P L
    qerr = abs(Q.conj().T @ Q - np.eye(r)).max()
    aerr = abs(X - Af).max() / abs(Af).max()
    merr = abs(M - Ri @ Q.conj().T).max() / abs(M).max()
    v = rng.standard_normal(n) + (0 if real else 1j * rng.standard_normal(n))
    b = A @ v
    z = np.zeros(n, complex)
    z[piv] = M.conj().T @ (M @ b[piv])
    res = np.linalg.norm(A @ z - b) / np.linalg.norm(b)
    print(f"min-norm operator n={n} rank {r} real={real}: |Q^H Q - I| {qerr:.1e}, rel |QR - PL| "
          f"{aerr:.1e}, |M - R^-1 Q^H| {merr:.1e}, residual {res:.1e}, |z|/|v| "
          f"{np.linalg.norm(z) / np.linalg.norm(v):.3f}")
    assert qerr < 1e-12 and aerr < 1e-6 and merr < 1e-12
    assert res < 1e-6 and np.linalg.norm(z) <= np.linalg.norm(v)
    if real:
        assert abs(M.imag).max() == 0.0


@pytest.mark.parametrize("kmesh,npts", [((1, 1, 3), 24), ((3, 1, 2), 24), ((2, 3, 1), 24),
                                        ((4, 4, 4), 24), ((4, 4, 4), 200)])
def test_build_y_kmesh_paths(env, kmesh, npts):
    """fisdf_build_y on the generic LDS k-mesh kernel ((1,1,3), (3,1,2), (2,3,1)) and the
    register / fused one (4x4x4; 200 points = 13 I-tiles, more than one I-group of the fused
    kernel's tile order, the last one partial), with fx stored for every k and for the
    time-reversal representatives k <= -k only (fisdf_set_time_reversal), against the oracle's
    y (fftisdf.py:73-85)."""
    torch, L, ctx = env
    import os, sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import isdf_ref as R
    from fisdf import cell as Cm
    cell = Cm.toy_cell(mesh=(6, 6, 6))
    coords = cell.gen_uniform_grids(cell.mesh)
    chi = Cm.eval_ao_kpts(cell, coords, kmesh)            # (nk, ngrid, nao)
    nk, ngrid, nao = chi.shape
    pts = np.random.default_rng(5).choice(ngrid, npts, replace=False)
    xip = np.ascontiguousarray(chi[:, pts, :])
    phase = R.get_phase(cell.a, R.get_kpts(cell.a, kmesh), kmesh)
    ref = R.build_y(chi, xip, phase)                       # (nk, ngrid, nip)
    nip = xip.shape[1]
    f, X = dev(torch, chi), dev(torch, xip)
    yT = torch.zeros((nk, nip, ngrid), dtype=torch.complex128, device="cuda")
    km = (C.c_int * 3)(*kmesh)
    a = (C.c_double * 9)(*cell.a.ravel())
    h = ngrid // 3
    for tr in (0, 1):
        ctx.call("fisdf_set_time_reversal", tr)
        yT.zero_()
        for g0, g1 in ((0, h), (h, ngrid)):  # two blocks: the g0 offset
            ctx.call("fisdf_build_y", C.c_void_p(f.data_ptr() + g0 * nao * 16), ngrid * nao, g0,
                     g1 - g0, ngrid, L.ptr(X), nip, nao, km, a, 0, nk, L.ptr(yT))
        torch.cuda.synchronize()
        y = yT.cpu().numpy().transpose(0, 2, 1)
        rel = abs(y - ref).max() / abs(ref).max()
        print(f"kmesh {kmesh} time_reversal={tr}: max rel |y - y_oracle| = {rel:.2e}")
        assert rel < 1e-12
    ctx.call("fisdf_set_time_reversal", 0)


@pytest.mark.parametrize("n", [1, 17, 36, 44, 64, 65, 81, 100, 128, 145, 236])
def test_cholesky_unpivoted_partial_blocks(env, n):
    """fisdf_cholesky (the fit's unpivoted blocked Cholesky: 64-column blocks, diagonal blocks
    factored and 16x16-block inverted in LDS, panel by the block inverse^H, HERK trailing update)
    vs numpy on random Hermitian PD matrices whose size leaves a partial last block (n % 64 in
    {1, 17, 36, 44, 0, ...}); batch of 3, one with a diagonal block of condition ~1e10."""
    torch, L, ctx = env
    rng = np.random.default_rng(100 + n)
    batch = 3
    A = np.empty((batch, n, n), complex)
    for b in range(batch):
        B = rnd(rng, n, n + 8)
        if b == 2:  # ill-conditioned: a geometric spectrum over 1e10 (every 64-block sees it)
            Q, _ = np.linalg.qr(rnd(rng, n, n))
            A[b] = (Q * np.logspace(0, -10, n)) @ Q.conj().T
        else:
            A[b] = B @ B.conj().T / n + np.eye(n)
        A[b] = 0.5 * (A[b] + A[b].conj().T)
    dA = dev(torch, A)
    fail = np.zeros(batch, np.int32)
    ctx.call("fisdf_cholesky", L.ptr(dA), n, batch, 1e-14, fail.ctypes.data_as(L._ip))
    assert (fail == 0).all(), fail
    out = dA.cpu().numpy()
    for b in range(batch):
        Lg = np.tril(out[b])
        Lr = np.linalg.cholesky(A[b])
        rel = abs(Lg - Lr).max() / abs(Lr).max()
        res = abs(Lg @ Lg.conj().T - A[b]).max() / abs(A[b]).max()
        print(f"n={n} b={b}: rel |L - L_np| {rel:.1e}, rel |L L^H - A| {res:.1e}")
        assert res < 1e-13
        # forward error bounded by the conditioning of the factor
        assert rel < (1e-12 if b < 2 else 1e-4)


@pytest.mark.parametrize("n", [300, 600])
def test_tri_inverse_batch_invariant(env, n):
    """L^{-1} by the factor stage's merged block-row substitution (split-K on the long block rows
    for nip >= 256): a matrix inverted alone equals, bit for bit, the same matrix inverted inside
    a batch of 8 (the k-sharded build factors fewer q per call than the 1-GPU build),
    and matches numpy to the conditioning."""
    torch, L, ctx = env
    rng = np.random.default_rng(n)
    batch = 8
    Ls = np.tril(rnd(rng, batch, n, n)) * 0.3 / np.sqrt(n)
    for b in range(batch):
        Ls[b][np.diag_indices(n)] = 1.0 + rng.random(n)
    dL = dev(torch, Ls)
    dI = torch.empty_like(dL)
    ctx.call("fisdf_tri_inverse", L.ptr(dL), n, batch, L.ptr(dI))
    inv_b = dI.cpu().numpy()
    for b in (0, 5):
        d1 = dev(torch, Ls[b:b + 1])
        o1 = torch.empty_like(d1)
        ctx.call("fisdf_tri_inverse", L.ptr(d1), n, 1, L.ptr(o1))
        one = o1.cpu().numpy()[0]
        assert np.array_equal(one, inv_b[b]), abs(one - inv_b[b]).max()
        ref = np.linalg.inv(Ls[b])
        rel = abs(inv_b[b] - ref).max() / abs(ref).max()
        assert rel < 1e-12, rel


@pytest.mark.parametrize("M,N,K,mode,beta", [
    (600, 1000, 600, 0, 0), (600, 1000, 600, 4, 0), (600, 777, 600, 5, 0), (600, 600, 600, 1, 0),
    (24, 700, 50, 0, 0), (100, 2000, 33, 0, 0), (1, 512, 8, 0, 0), (129, 513, 17, 4, 0),
    (64, 4096, 64, 5, 0), (600, 24624, 600, 5, 0),
    # beta != 0: the read-modify-write epilogue (trsm_blocked's trailing update B -= L X runs
    # through this kernel with beta = 1, FULL or A_REAL)
    (64, 1024, 128, 0, 1), (100, 777, 64, 1, 1), (33, 2048, 40, 0, 2), (600, 600, 200, 1, 2)])
def test_zgemm_modes_wide(env, M, N, K, mode, beta):
    """NN products through fisdf_zgemm_mode: N >= 512 takes the 64 x 128-tile kernel
    (zgemm_wide.hip) — FULL (3 MFMAs per complex block), A_REAL (Im A ignored), A_LOWER (K loop
    cut at each M-tile's last row) and both, M-edge tiles with <= 32 rows, ragged N, beta = 0, 1
    or complex with a nonzero C — against numpy on the matrices the mode describes."""
    torch, L, ctx = env
    rng = np.random.default_rng(M * 7 + N + K + mode)
    A, B = rnd(rng, M, K), rnd(rng, K, N)
    Aeff = A.copy()
    if mode & 1:
        Aeff = Aeff.real.astype(complex)
    if mode & 4:
        Aeff = np.tril(Aeff)
        # lower triangular input; past each 64-row M-tile's last row the K loop stops, so
        # anything there must never be read
        beyond = np.arange(K)[None, :] >= 64 * (np.arange(M)[:, None] // 64 + 1)
        A = np.tril(A) + np.where(beyond, rnd(rng, M, K) * 1e3, 0)
    dA, dB = dev(torch, A), dev(torch, B)
    C0 = rnd(rng, M, N) if beta else np.zeros((M, N), complex)
    dC = dev(torch, C0)
    bv = {0: 0.0, 1: 1.0, 2: -0.5 + 0.25j}[beta]
    one, vb = np.array([1.0, 0.0]), np.array([bv.real, bv.imag]) if beta else np.zeros(2)
    ctx.call("fisdf_zgemm_mode", 0, 0, M, N, K, one.ctypes.data_as(L._dp), L.ptr(dA), K, 0,
             L.ptr(dB), N, 0, vb.ctypes.data_as(L._dp), L.ptr(dC), N, 0, 1, mode)
    ref = Aeff @ B + (bv * C0 if beta else 0)
    err = abs(dC.cpu().numpy() - ref).max()
    assert err < 1e-12 * max(K, 16), err
