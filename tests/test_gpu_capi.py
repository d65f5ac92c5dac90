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


def _device_count():
    import torch
    return torch.cuda.device_count()


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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode,size,name,variant", [
    ("host", 2, "toy222", ""), ("host", 3, "toy331_fr", ""), ("rccl", 1, "toy222", ""),
    ("host", 2, "toy331_fr", "svd"), ("host", 3, "toy222", "notr"),
    ("host", 6, "toy331_fr", ""),    # 5 fitted q on 6 ranks: one rank fits none
    ("group", 3, "toy331_fr", ""), ("group", 2, "toy222", "notr"), ("group", 1, "toy222", "rccl"),
    ("group", 2, "toy331_fr", "multidev"), ("group", 2, "toy331_fr", "multidev_rccl")])
def test_capi_build_sharded(mode, size, name, variant):
    """fisdf_build_sharded (SURVEY §8(e) through the C-ABI, no torch): SIZE ranks on GPU 0
    (tests/capi_shard_worker.py), the collectives from the caller (host: a file mailbox per
    collective, uneven q shares at 3 ranks; rccl: the library's RCCL fisdf_comm on a 1-rank
    communicator).  Every rank's W_q equal the 1-GPU build's bit for bit, every rank holds W_0,
    the W_s row blocks are the 1-GPU W_s rows, and the all-reduced J/K of every rank equal the
    1-GPU get_jk to rounding.  Variants: fit="svd" (the minimum-norm operator on every q) and
    time reversal off (all nk q fitted and shared).  group: every rank in one process through
    fisdf_group (SURVEY §8(b)'s multi-device handle: a thread and a stream per rank, the
    collectives as device copies between the ranks' buffers); multidev: rank r on GPU r (device
    copies across xGMI, or RCCL with 2 ranks), skipped where fewer GPUs are visible."""
    if variant.startswith("multidev") and _device_count() < size:
        pytest.skip(f"needs {size} GPUs (one rank per device)")
    with tempfile.TemporaryDirectory() as tmp:
        nproc = 1 if mode == "group" else size   # group: all ranks in one process (fisdf_group)
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "capi_shard_worker.py"), name,
                                   str(r), str(size), tmp, mode, variant]) for r in range(nproc)]
        rcs = []
        for p in procs:
            try:
                rcs.append(p.wait(timeout=240))
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert rcs == [0] * nproc, rcs
        outs = [dict(np.load(os.path.join(tmp, f"rank{r}.npz"))) for r in range(size)]
    ref = outs[0]
    qs = np.concatenate([o["fit_qs"] for o in outs])
    assert sorted(qs.tolist()) == ref["ref_fit_qs"].tolist()
    slot = {int(q): i for i, q in enumerate(ref["ref_fit_qs"])}
    lo = 0
    for r, o in enumerate(outs):
        assert np.array_equal(o["perm"], ref["perm"])              # replicated selection
        for i, q in enumerate(o["fit_qs"]):
            assert np.array_equal(o["wq"][i], ref["ref_wq"][slot[int(q)]]), (r, q)
        assert np.array_equal(o["w0"], ref["ref_wq"][0])
        i0, i1 = o["rows"]
        assert i0 == lo
        lo = i1
        dws = abs(o["ws_rows"] - ref["ref_ws"][:, i0:i1]).max()
        assert dws < 1e-12 * max(1.0, abs(ref["ref_ws"]).max()), dws
        dj, dk = abs(o["vj"] - ref["ref_vj"]).max(), abs(o["vk"] - ref["ref_vk"]).max()
        print(f"\n{name} {mode}{' ' + variant if variant else ''} rank {r}/{size}: "
              f"q {o['fit_qs'].tolist()} rows [{i0}, {i1}) "
              f"|dWs| {dws:.1e} |dJ| {dj:.1e} |dK| {dk:.1e} vs the 1-GPU build")
        assert dj < 1e-11 and dk < 1e-11
        assert np.array_equal(o["vj"], outs[0]["vj"]) and np.array_equal(o["vk"], outs[0]["vk"])
        if mode == "host":   # a2a per local q, one reduce-scatter, one broadcast, J + K
            n_a2a = max(len(x["fit_qs"]) for x in outs)
            assert o["calls"].tolist() == [n_a2a, 2, 1, 1], o["calls"]  # sorted names
    assert lo == ref["perm"].size
