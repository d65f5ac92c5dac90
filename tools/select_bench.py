"""The C3 selection alone (fisdf_select_points: real-part Gram + pivoted Cholesky + one pinned
read-back), ms per call and per pivot; FISDF_SEL_MODE picks the kernel (batch / coop / blocked).
  python tools/select_bench.py [--cfg c3] [--reps 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fisdf import _lib as L  # noqa: E402
from fisdf import cell as C  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="c3")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--save", default=None, help="write the pivots (npz) to compare selection modes")
a = ap.parse_args()
kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS[a.cfg]
cell = {"diamond": C.diamond_cell, "nio": C.nio_cell, "si": C.si_supercell}[kind](basis=basis, mesh=mesh)
nao = cell.nao_nr()
x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
nk, ng0 = x0.shape[0], x0.shape[1]
ctx = L.Context(0, torch.cuda.current_stream().cuda_stream)
dx = torch.from_numpy(np.ascontiguousarray(x0)).cuda()
perm = np.zeros(nip, np.int32)
npiv = L.C.c_int()
full = L.C.c_int()


def run():
    ctx.call("fisdf_select_points", L.ptr(dx), nk, ng0, nao, nip, 0.0,
             perm.ctypes.data_as(L._ip), L.C.byref(npiv), L.C.byref(full))


run()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.reps):
    run()
ms = (time.perf_counter() - t) / a.reps * 1e3
print(f"select {a.cfg} ng0 {ng0} nip {nip} mode {os.environ.get('FISDF_SEL_MODE', 'batch')}: "
      f"{ms:.3f} ms per call, {npiv.value} pivots "
      f"({ms / max(npiv.value, 1) * 1e3:.2f} us per pivot incl. Gram)", flush=True)
if a.save:
    np.savez(a.save, perm=perm[:min(nip, npiv.value)].copy())
