"""Simulate the batched-candidate pivoted Cholesky: how many exact greedy steps run on a
candidate set (top-m residual diagonals) before a non-candidate could win."""
import sys, time
import numpy as np
import os; _R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0] = [_R, os.path.join(_R, "fft-isdf-scratch_amd")]
from fisdf import cell as C
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
import bench
kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS[cfg]
make = {"diamond": C.diamond_cell, "nio": C.nio_cell, "si": C.si_supercell}[kind]
cell = make(basis=basis, mesh=mesh)
t = time.time()
x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
nk = x0.shape[0]
x2 = np.zeros((x0.shape[1],) * 2)
for k in range(nk):
    x2 += (x0[k].conj() @ x0[k].T).real
x4 = x2 * x2 / nk
print("x4", x4.shape, time.time() - t, flush=True)
n = x4.shape[0]
d0 = np.diag(x4).copy()
# plain greedy
L = np.zeros((n, nip)); d = d0.copy(); piv = []
for j in range(nip):
    p = int(np.argmax(d)); piv.append(p)
    col = (x4[:, p] - L[:, :j] @ L[p, :j]) / np.sqrt(d[p]); L[:, j] = col; d = d - col * col; d[piv] = -1
piv = np.array(piv)
for m in (16, 32, 64, 128, 256):
    # batches: candidates = top-m of d (excluding chosen), bound B = (m+1)th largest
    d = d0.copy(); j = 0; batches = 0; dd = d0.copy()
    chosen = np.zeros(n, bool)
    while j < nip:
        # residual diag at step j (exact)
        dd = d0 - (L[:, :j] ** 2).sum(1); dd[chosen] = -np.inf
        order = np.argsort(-dd, kind="stable")
        cand = order[:m]; B = dd[order[m]] if m < n else -np.inf
        cset = set(cand.tolist())
        s = 0
        while j < nip:
            p = piv[j]
            if p not in cset: break
            # at step j the greedy pick p must beat every non-candidate's (upper-bound) residual
            if not (dd_now := d0[p] - (L[p, :j] ** 2).sum()) > B: break
            chosen[p] = True; j += 1; s += 1
        batches += 1
        if s == 0:  # fall back: one plain step
            chosen[piv[j]] = True; j += 1
    print(f"m={m}: {batches} batches for {nip} pivots ({nip / batches:.1f} per batch)", flush=True)
