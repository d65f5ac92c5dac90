"""The RCCL code path on the one GPU the pool gives ("an RCCL loop-back on a
single device"): a one-rank ``nccl`` group forces ISDF through its multi-GPU branch (chunked
all-to-all of y, W_s all-reduce, W_0 broadcast, get_jk all-reduces; kshard.py) and the result
must equal the plain one-GPU build — W_q bit for bit (same kernels, same per-q arithmetic),
J/K (incl. exxdiv='ewald' and omega) to <= 1e-12."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["toy333_fr", "toy222"])
def test_rccl_sharded_path_matches_plain(name):
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "r.npz")
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
        p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py"), name, out],
                           env=env, timeout=300)
        assert p.returncode == 0
        o = dict(np.load(out))
    assert str(o["backend"]) == "nccl"
    assert np.array_equal(o["plain_perm"], o["rccl_perm"])
    assert np.array_equal(o["plain_wq"], o["rccl_wq"]), "RCCL path changed W_q"
    scale = max(1.0, abs(o["plain_vk"]).max(), abs(o["plain_vj"]).max())
    for k in ("vj", "vk", "vke", "vjw", "vkw"):
        d = abs(o[f"plain_{k}"] - o[f"rccl_{k}"]).max()
        print(f"{name}: RCCL vs plain |d{k}| = {d:.1e}")
        assert d <= 1e-12 * scale, (k, d)


@pytest.mark.parametrize("name,n", [("toy333_fr", 3), ("toy331", 2)])
def test_emulated_rank_reproduces_its_q(name, n):
    """bench.py --emulate-ranks times each rank's share of an N-rank build on one GPU
    (kshard.EmulatedGroup: the all-to-all pieces handed over from a full 1-GPU y).  Its arithmetic
    is the sharded build's: every emulated rank's W_q of its own q equal the 1-GPU W_q bit for bit,
    and its W_s rows are the partial sum of its own q (the reduce-scatter's local input)."""
    import torch
    from cases import inputs
    from fisdf import ISDF, kshard, _lib
    from fisdf.isdf import _fit_qset
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    df1 = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    d = df1.device
    df1._kmesh()
    df1._ao_parent = d.to_dev(x0)
    df1._ao_grid = d.to_dev(chi)
    df1.build()
    wq1 = df1._wq
    X = df1._dev_state["X"]
    nk, nip, nao = X.shape
    ngrid = chi.shape[1]
    fit_qs, partner, _ = _fit_qset(df1, np.asarray(kmesh))
    qs = np.ascontiguousarray(fit_qs, dtype=np.int32)
    yall = d.empty((len(qs), nip, ngrid))
    km_c, km_p = _lib.iarr(kmesh)
    a_c, a_p = _lib.darr(cell.a.ravel())
    # the 1-GPU build's y arithmetic (fisdf_build restores the context's stage settings on return)
    d.ctx.call("fisdf_set_time_reversal", 1 if df1.time_reversal_used else 0)
    d.ctx.call("fisdf_build_y_qs", _lib.ptr(df1._ao_grid), ngrid * nao, 0, ngrid, ngrid,
               _lib.ptr(X), nip, nao, km_p, a_p, qs.ctypes.data_as(_lib._ip), len(qs),
               _lib.ptr(yall))
    real_q = np.array([partner[q] == q for q in fit_qs])
    chunks = kshard.assign_q(np.where(real_q, 0.6, 1.0), n)
    slices = kshard.grid_slices(cell.mesh, n)
    for R in range(n):
        df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0,
                  comm=kshard.EmulatedGroup(R, n, kshard.emulated_pieces(yall, chunks, slices, R)))
        df._kmesh()
        df._ao_parent, df._ao_grid = df1._ao_parent, df1._ao_grid
        df.build()
        df.get_jk(dm)
        assert np.array_equal(df.perm, df1.perm)
        wq = df._dev_state["Wq"].cpu().numpy()
        for j, q in enumerate(df.my_qs):
            assert np.array_equal(wq[j], wq1[q]), (R, q, abs(wq[j] - wq1[q]).max())
        print(f"{name} emulated rank {R}/{n}: q {list(df.my_qs)} W_q bitwise equal to 1-GPU")
    torch.cuda.synchronize()
