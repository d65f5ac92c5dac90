"""Worker of tests/test_gpu_rccl.py: the collective (k-sharded) code path over RCCL on ONE GPU.

Run as  RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/rccl_worker.py
        <case> <out.npz>
A one-rank ``nccl`` group (RCCL) with ``ISDF.force_sharded``: the build takes the multi-GPU
branch — grid-sliced y, the per-q chunked RCCL all-to-all (async, stream-ordered waits), the
unpack + ready marks feeding one fit call, the real-part W_s all-reduce and the W_0 broadcast —
and get_jk its row-block contraction + all-reduces (fftisdf.py:97-122, 204-207, 133-228)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), HERE]

import numpy as np  # noqa: E402


def main():
    name, out = sys.argv[1], sys.argv[2]
    import torch
    import torch.distributed as dist
    from cases import inputs
    from fisdf import ISDF
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    res = {}
    for tag, comm, forced in (("plain", None, False), ("rccl", dist.group.WORLD, True)):
        df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0, device=0, comm=comm)
        df.force_sharded = forced
        d = df.device
        df._kmesh()
        df._ao_parent = d.to_dev(x0)
        df._ao_grid = d.to_dev(chi)
        df.build()
        vj, vk = df.get_jk(dm)
        _, vke = df.get_jk(dm, exxdiv="ewald")
        vjw, vkw = df.get_jk(dm, omega=0.4)
        res.update({f"{tag}_{k}": v for k, v in dict(vj=vj, vk=vk, vke=vke, vjw=vjw, vkw=vkw,
                                                     wq=df._wq, perm=df.perm).items()})
        torch.cuda.synchronize()
        del df
    np.savez(out, backend=dist.get_backend(), **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
