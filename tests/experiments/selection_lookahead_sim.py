"""Lookahead-1 selection: per exchange the top-3 residual diagonals (p, q, T); after pivot p's
column, if d'_q > T then q is the next greedy pivot without another exchange."""
import sys, time
import numpy as np
import os; _R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0] = [_R, os.path.join(_R, "fft-isdf-scratch_amd")]
from fisdf import cell as C
import bench
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS[cfg]
make = {"diamond": C.diamond_cell, "nio": C.nio_cell, "si": C.si_supercell}[kind]
cell = make(basis=basis, mesh=mesh)
x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
nk = x0.shape[0]
x2 = np.zeros((x0.shape[1],) * 2)
for k in range(nk):
    x2 += (x0[k].conj() @ x0[k].T).real
x4 = x2 * x2 / nk
n = x4.shape[0]
L = np.zeros((n, nip)); d = np.diag(x4).copy(); j = 0; ex = 0; two = 0
chosen = np.zeros(n, bool)
def step(p, j):
    col = (x4[:, p] - L[:, :j] @ L[p, :j]) / np.sqrt(d[p]); L[:, j] = col
    return col
while j < nip:
    dd = np.where(chosen, -np.inf, d)
    order = np.argsort(-dd, kind="stable")
    p, q, t = order[0], order[1], dd[order[2]]
    ex += 1
    col = step(p, j); d -= col * col; chosen[p] = True; j += 1
    if j < nip and d[q] > t:
        # q is the exact next pivot: every other row's residual <= its old value <= t
        dd2 = np.where(chosen, -np.inf, d)
        assert int(np.argmax(dd2)) == q
        col = step(q, j); d -= col * col; chosen[q] = True; j += 1; two += 1
print(f"{cfg}: {nip} pivots in {ex} exchanges ({two} lookahead hits)")
