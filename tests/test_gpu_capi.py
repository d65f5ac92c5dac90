"""The composite C-ABI (fisdf_build / fisdf_get_jk / fisdf_get_wq, include/fisdf.h; SURVEY.md
§8(b)) driven without torch (tests/capi_worker.py: ctypes + NumPy, fisdf_malloc and
fisdf_memcpy_* for every buffer), against the oracle (the reference's CPU path, fftisdf.py:22-228
with gelsy and dpstrf, restated): same interpolation points, J/K of a two-matrix dm set
(nset = 2, the KUHF shape; fftisdf.py:155,166,210) < 1e-8 Ha, and _x / _w0 / _wq as the
reference's attributes (fftisdf.py:125-128)."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["toy222", "toy333_fr"])
def test_capi_build_get_jk_torch_free(name):
    from cases import inputs, oracle
    from oracle import isdf_ref as R
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "c.npz")
        p = subprocess.run([sys.executable, os.path.join(HERE, "capi_worker.py"), name, out],
                           timeout=240)
        assert p.returncode == 0
        o = dict(np.load(out))
    assert int(o["torch_loaded"]) == 0
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    ref = oracle(name)
    same = np.array_equal(o["perm"], ref["perm"])
    if not same:   # a tie-certified selection (test_gpu_selection.py): the oracle on these points
        ref = dict(xip=x0[:, o["perm"]])
        ref.update(R.build(ref["xip"], chi, coords, cell.a, kmesh, cell.mesh))
    print(f"\n{name}: C-ABI selection {'identical to' if same else 'tie-certified against'} dpstrf")
    assert np.array_equal(o["x"], x0[:, o["perm"]])                         # _x (:125)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    xip = ref["xip"]
    dms = o["dms"]
    vj0 = R.get_j_kpts(xip, ref["w0"], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk0 = R.get_k_kpts(xip, ref["wq"], dms, phase)
    dj, dk = abs(o["vj"] - vj0).max(), abs(o["vk"] - vk0).max()
    print(f"{name}: C-ABI (no torch) nip {len(o['perm'])} fitted q {int(o['nfit'])} "
          f"(min-norm {int(o['min_norm'])}), nset 2: |dJ| {dj:.2e} |dK| {dk:.2e} Ha")
    assert dj < 1e-8 and dk < 1e-8
    # nset = 2 is two independent get_jk: each set equals its own single-set result
    for x in range(2):
        assert abs(o["vk"][x] - vk0[x]).max() < 1e-8
    # _wq: the fitted q and their time-reversal partners conj(W_q), W_0 = _wq[0] (:126-128)
    assert np.array_equal(o["w0"], o["wq"][0])
    nk = int(np.prod(kmesh))
    v = np.stack(np.unravel_index(np.arange(nk), tuple(kmesh)), 1)
    mv = (-v) % np.asarray(kmesh)
    partner = (mv[:, 0] * kmesh[1] + mv[:, 1]) * kmesh[2] + mv[:, 2]
    for q in range(nk):
        if partner[q] != q:
            assert np.array_equal(o["wq"][partner[q]], o["wq"][q].conj())
