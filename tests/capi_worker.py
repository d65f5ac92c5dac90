"""Drive libfisdf.so through its composite C entries only — ctypes + NumPy, no torch in the
process (tests/test_gpu_capi.py runs this as a subprocess and asserts it).  What a C, Fortran or
cffi caller of include/fisdf.h does: fisdf_create on the null stream, fisdf_malloc /
fisdf_memcpy_* for every device buffer, fisdf_build (the reference's ISDF.build(), fftisdf.py:
308-325), fisdf_get_jk with nset = 2 density matrices (a KUHF-shaped (2, nk, nao, nao) set,
fftisdf.py:210), fisdf_get_x / _w0 / _wq, and the per-context error message.

usage: python capi_worker.py CASE OUT.npz
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

from fisdf import _lib  # noqa: E402
from fisdf import cell as Cl  # noqa: E402


def main(case, out):
    from cases import inputs
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(case)
    nk, nao = int(np.prod(kmesh)), cell.nao_nr()
    dms = np.concatenate([dm, Cl.make_dm(nao, kmesh, cell, seed=99, scale=0.2)[None]])  # (2, nk, nao, nao)
    lib = _lib.load()
    ctx = C.c_void_p()
    rc = lib.fisdf_create(0, None, C.byref(ctx))
    assert rc == 0, lib.fisdf_last_error(None)

    def call(name, *args):
        rc = getattr(lib, name)(ctx, *args)
        if rc != 0:
            raise RuntimeError(f"{name}: {lib.fisdf_last_error(ctx).decode()}")

    def upload(a):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        call("fisdf_malloc", C.c_size_t(a.nbytes), C.byref(p))
        call("fisdf_memcpy_htod", p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes))
        return p

    def alloc(nbytes):
        p = C.c_void_p()
        call("fisdf_malloc", C.c_size_t(nbytes), C.byref(p))
        return p

    d_x0, d_f, d_dms = upload(x0), upload(chi), upload(dms.astype(np.complex128))
    km, kp = _lib.iarr(kmesh)
    me, mp = _lib.iarr(cell.mesh)
    aa, ap = _lib.darr(cell.a.ravel())
    opts = _lib.BuildOpts()
    lib.fisdf_build_opts_default(C.byref(opts))
    opts.nip_max = int(nao * c0)                                           # fftisdf.py:383
    nip = C.c_int()
    call("fisdf_build", d_x0, x0.shape[1], d_f, nao, kp, mp, ap, C.byref(opts), C.byref(nip))
    r = _lib.BuildResult()
    call("fisdf_build_get", C.byref(r))
    nip = nip.value
    assert r.nip == nip and r.nk == nk and r.nao == nao
    perm = np.ctypeslib.as_array(r.perm, (nip,)).copy()
    ranks = np.ctypeslib.as_array(r.ranks, (r.nfit,)).copy()
    nbytes = dms.size * 16
    d_vj, d_vk = alloc(nbytes), alloc(nbytes)
    call("fisdf_get_jk", d_dms, 2, 1, 1, d_vj, d_vk)
    vj = np.empty(dms.shape, complex)
    vk = np.empty(dms.shape, complex)
    call("fisdf_memcpy_dtoh", vj.ctypes.data_as(C.c_void_p), d_vj, C.c_size_t(nbytes))
    call("fisdf_memcpy_dtoh", vk.ctypes.data_as(C.c_void_p), d_vk, C.c_size_t(nbytes))
    hx = np.empty((nk, nip, nao), complex)
    hw0 = np.empty((nip, nip), complex)
    hwq = np.empty((nk, nip, nip), complex)
    call("fisdf_get_x", hx.ctypes.data_as(C.c_void_p))
    call("fisdf_get_w0", hw0.ctypes.data_as(C.c_void_p))
    call("fisdf_get_wq", hwq.ctypes.data_as(C.c_void_p))
    # the error of one context is that context's: a second context asked for get_jk before any
    # build fails with its own message, the first context's message is untouched
    ctx2 = C.c_void_p()
    assert lib.fisdf_create(0, None, C.byref(ctx2)) == 0
    before = lib.fisdf_last_error(ctx)
    assert lib.fisdf_get_jk(ctx2, d_dms, 2, 1, 1, d_vj, d_vk) != 0
    err2 = lib.fisdf_last_error(ctx2).decode()
    assert "no build" in err2, err2
    assert lib.fisdf_last_error(ctx) == before
    assert lib.fisdf_destroy(ctx2) == 0
    # a failed fisdf_create reports through fisdf_last_error(NULL) and leaves every live
    # context's message alone
    ctx3 = C.c_void_p()
    assert lib.fisdf_create(1 << 20, None, C.byref(ctx3)) != 0
    assert b"device id" in lib.fisdf_last_error(None)
    assert lib.fisdf_last_error(ctx) == before
    assert r.time_reversal == 1 and r.tr_deviation < 1e-12, (r.time_reversal, r.tr_deviation)
    for p in (d_x0, d_f, d_dms, d_vj, d_vk):
        call("fisdf_free", p)
    call("fisdf_build_release")
    assert lib.fisdf_destroy(ctx) == 0
    assert "torch" not in sys.modules, "the C-ABI path must not need torch"
    np.savez(out, perm=perm, ranks=ranks, vj=vj, vk=vk, x=hx, w0=hw0, wq=hwq, dms=dms,
             nfit=r.nfit, min_norm=r.min_norm_slots, err2=err2, torch_loaded=0)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
