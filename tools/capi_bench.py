"""C3 build + get_jk through the composite C-ABI only (fisdf_build / fisdf_get_jk), in a process
that never imports torch: one HIP runtime (the system ROCm's) in the address space.  Used (i) to
time the library's own orchestration without the Python mirror and (ii) under rocprofv3, to see
whether the profiled process exits cleanly when torch's bundled HIP runtime is absent (the exit-
time SIGSEGV of DESIGN §6 is in torch's libamdhip64 teardown).

usage: python tools/capi_bench.py [--config c3] [--steps 10] [--warmup 2]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import bench
    from fisdf import _lib
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup(args.config)
    nk, nao = int(np.prod(kmesh)), cell.nao_nr()
    lib = _lib.load()
    ctx = C.c_void_p()
    assert lib.fisdf_create(0, None, C.byref(ctx)) == 0, lib.fisdf_last_error(None)

    def call(name, *a):
        if getattr(lib, name)(ctx, *a) != 0:
            raise RuntimeError(lib.fisdf_last_error(ctx).decode())

    def upload(a):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        call("fisdf_malloc", C.c_size_t(a.nbytes), C.byref(p))
        call("fisdf_memcpy_htod", p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes))
        return p

    d_x0, d_f = upload(x0), upload(chi)
    del chi
    dms = dm[None].astype(np.complex128)
    d_dms = upload(dms)
    d_vj, d_vk = upload(np.zeros_like(dms)), upload(np.zeros_like(dms))
    km, kp = _lib.iarr(kmesh)
    me, mp = _lib.iarr(cell.mesh)
    aa, ap_ = _lib.darr(cell.a.ravel())
    opts = _lib.BuildOpts()
    lib.fisdf_build_opts_default(C.byref(opts))
    opts.nip_max = int(nao * c0)
    nip = C.c_int()

    def step():
        call("fisdf_build", d_x0, x0.shape[1], d_f, nao, kp, mp, ap_, C.byref(opts), C.byref(nip))
        call("fisdf_get_jk", d_dms, 1, 1, 1, d_vj, d_vk)

    for _ in range(args.warmup):
        step()
    call("fisdf_sync")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    call("fisdf_sync")
    dt = (time.perf_counter() - t0) / args.steps
    vk = np.empty(dms.shape, complex)
    call("fisdf_memcpy_dtoh", vk.ctypes.data_as(C.c_void_p), d_vk, C.c_size_t(vk.nbytes))
    for p in (d_x0, d_f, d_dms, d_vj, d_vk):
        call("fisdf_free", p)
    call("fisdf_build_release")
    lib.fisdf_destroy(ctx)
    print(json.dumps({"driver": "composite C-ABI (fisdf_build + fisdf_get_jk), no torch",
                      "config": args.config, "nip": nip.value, "steps": args.steps,
                      "ms_per_step": round(dt * 1e3, 3), "k_points_per_s": round(nk / dt, 3),
                      "max_abs_vk": float(abs(vk).max()),
                      "torch_loaded": "torch" in sys.modules}))


if __name__ == "__main__":
    main()
