"""Case files and the oracle check of the host-AddressSanitizer C-ABI run (tools/asan_check.sh).

  python tools/asan/check.py make CASE DIR     writes DIR/case.bin (tests/cases.py inputs, nset 2)
  python tools/asan/check.py verify CASE DIR   reads DIR/out.bin (tools/asan/capi_asan) and checks
                                               J/K against the oracle (fftisdf.py:133-228
                                               restated) < 1e-8 Ha, as tests/test_gpu_capi.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

MAGIC = 0x44534946


def _dms(name):
    from cases import inputs
    from fisdf import cell as Cl
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    extra = Cl.make_dm(cell.nao_nr(), kmesh, cell, seed=99, scale=0.2)[None]
    return np.ascontiguousarray(np.concatenate([dm, extra]).astype(np.complex128))


def make(name, d):
    from cases import inputs
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    nk, nao = int(np.prod(kmesh)), cell.nao_nr()
    dms = _dms(name)
    hdr = np.array([MAGIC, nk, x0.shape[1], chi.shape[1], nao, int(nao * c0), dms.shape[0],
                    *kmesh, *cell.mesh, 0], np.int32)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "case.bin"), "wb") as f:
        f.write(hdr.tobytes())
        f.write(np.ascontiguousarray(cell.a, np.float64).ravel().tobytes())
        for arr in (x0, chi, dms):
            f.write(np.ascontiguousarray(arr, np.complex128).tobytes())


def verify(name, d):
    from cases import inputs, oracle
    from oracle import isdf_ref as R
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    nk, nao = int(np.prod(kmesh)), cell.nao_nr()
    dms = _dms(name)
    raw = open(os.path.join(d, "out.bin"), "rb").read()
    nip = int(np.frombuffer(raw, np.int32, 1)[0])
    perm = np.frombuffer(raw, np.int32, nip, 4)
    off = 4 + 4 * nip
    vj = np.frombuffer(raw, np.complex128, dms.size, off).reshape(dms.shape)
    vk = np.frombuffer(raw, np.complex128, dms.size, off + 16 * dms.size).reshape(dms.shape)
    ref = oracle(name)
    if not np.array_equal(perm, ref["perm"]):   # a tie-certified selection: the oracle there
        ref = dict(xip=x0[:, perm])
        ref.update(R.build(ref["xip"], chi, coords, cell.a, kmesh, cell.mesh))
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    vj0 = R.get_j_kpts(ref["xip"], ref["w0"], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))
    vk0 = R.get_k_kpts(ref["xip"], ref["wq"], dms, phase)
    dj, dk = abs(vj - vj0).max(), abs(vk - vk0).max()
    print(f"{name}: host-ASan C-ABI run, nip {nip}, nset {dms.shape[0]}: |dJ| {dj:.2e} "
          f"|dK| {dk:.2e} Ha")
    assert dj < 1e-8 and dk < 1e-8


if __name__ == "__main__":
    {"make": make, "verify": verify}[sys.argv[1]](sys.argv[2], sys.argv[3])
