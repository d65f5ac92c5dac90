"""Worker for the multi-rank tests: one k-shard of the ISDF build + get_jk.

Run as  RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/dist_worker.py
        <case> <backend> <out.npz>
On the GPU pool several ranks share cuda:0 with the gloo backend (RCCL needs one GPU per
rank; the driver's 8-GPU bench exercises RCCL itself)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), HERE]

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402


def main():
    name, backend, out = sys.argv[1], sys.argv[2], sys.argv[3]
    import torch
    import torch.distributed as dist
    from cases import inputs, oracle
    from fisdf import ISDF
    dist.init_process_group(backend)
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0, device=0,
              comm=dist.group.WORLD)
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    if os.environ.get("FISDF_DIST_INJECT") == "1":
        df.set_interpolation_points(o["perm"])   # the oracle's (dpstrf) pivots
    df.build()
    vj, vk = df.get_jk(dm)
    vj0, vk0 = o["vj"], o["vk"]
    lanes, depth = C.c_int(), C.c_int()
    d.ctx.call("fisdf_fit_info", C.byref(lanes), C.byref(depth))
    extra = {}
    if os.environ.get("FISDF_DIST_EXTRAS") == "1":
        # next-4 in the sharded path: exxdiv='ewald' (the correction is added after the vk
        # all-reduce) and a range-separated refit (a collective build on every rank)
        from oracle import isdf_ref as R
        from fisdf.cell import madelung
        _, vk_e = df.get_jk(dm, exxdiv="ewald")
        # every reference below is the oracle on THIS build's interpolation points (df.perm),
        # whether or not they are dpstrf's: the checks hold on every run
        xip = x0[:, df.perm]
        kpts = R.get_kpts(cell.a, kmesh)
        phase = R.get_phase(cell.a, kpts, kmesh)
        if np.array_equal(df.perm, o["perm"]):
            vk_own = vk0
        else:
            ob0 = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh)
            vk_own = R.get_k_kpts(xip, ob0["wq"], dm, phase)
        S = np.einsum("kgm,kgn->kmn", chi.conj(), chi) * (cell.vol / chi.shape[1])
        vke0 = vk_own + madelung(cell, kmesh) * np.einsum("kmp,xkpq,kqn->xkmn", S, dm, S)
        vj_w, vk_w = df.get_jk(dm, omega=0.4)
        ob = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh, omega=0.4)
        extra = dict(vk_e=vk_e, vke0=vke0, vj_w=vj_w, vk_w=vk_w,
                     vjw0=R.get_j_kpts(xip, ob["w0"], dm), vkw0=R.get_k_kpts(xip, ob["wq"], dm, phase))
    np.savez(out, vj=vj, vk=vk, perm=df.perm, ranks=df.ranks, vj0=vj0, vk0=vk0,
             perm0=o["perm"], wq=df._wq, my_qs=df.my_qs, fit_lanes=lanes.value,
             fit_pipe=depth.value, y_streamed=bool(getattr(df, "y_streamed", False)), **extra)
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
