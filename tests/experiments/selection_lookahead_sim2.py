"""Lookahead-k selection: per exchange the top-(k+2) residual diagonals; pivots are accepted in
order while the next candidate's updated residual beats the bound (the (k+2)-th current value)."""
import sys
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
for K in (1, 2, 3, 4, 8):
    L = np.zeros((n, nip)); d = np.diag(x4).copy(); j = 0; ex = 0
    chosen = np.zeros(n, bool)
    while j < nip:
        dd = np.where(chosen, -np.inf, d)
        order = np.argsort(-dd, kind="stable")
        cands = list(order[:K + 1]); bound = dd[order[K + 1]]
        ex += 1
        for t, c in enumerate(cands):
            if t > 0:
                # candidate c must beat every non-candidate (<= bound) and the other candidates
                rest = [e for e in cands[t:] if e != c]
                if not (d[c] > bound and all(d[c] > d[e] or (d[c] == d[e] and c < e) for e in rest)):
                    break
            col = (x4[:, c] - L[:, :j] @ L[c, :j]) / np.sqrt(d[c]); L[:, j] = col
            d -= col * col; chosen[c] = True; j += 1
            if j >= nip: break
    print(f"{cfg} lookahead {K}: {nip} pivots in {ex} exchanges", flush=True)
