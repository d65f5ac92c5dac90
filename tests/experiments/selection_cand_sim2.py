"""Batch lengths of candidate rules on the C3 parent grid (exact greedy pivots given)."""
import sys, time
import numpy as np
import os; _R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0] = [_R, os.path.join(_R, "fft-isdf-scratch_amd")]
from fisdf import cell as C
import bench
kind, basis, mesh, kmesh, m0, nip = bench.CONFIGS["c3"]
cell = C.diamond_cell(basis=basis, mesh=mesh)
x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
x2 = sum((x0[k].conj() @ x0[k].T).real for k in range(x0.shape[0]))
x4 = x2 * x2 / x0.shape[0]
n = x4.shape[0]; d0 = np.diag(x4).copy()
L = np.zeros((n, nip)); d = d0.copy(); piv = []
for j in range(nip):
    p = int(np.argmax(d)); piv.append(p)
    col = (x4[:, p] - L[:, :j] @ L[p, :j]) / np.sqrt(d[p]); L[:, j] = col; d = d - col * col; d[piv] = -np.inf
piv = np.array(piv)
wave = (np.arange(n) % 512) // 64
def run(rule):
    j = 0; batches = 0; chosen = np.zeros(n, bool)
    while j < nip:
        dd = d0 - (L[:, :j] ** 2).sum(1); dd[chosen] = -np.inf
        cand, B = rule(dd)
        s = 0
        while j < nip and s < CAP and piv[j] in cand and (d0[piv[j]] - (L[piv[j], :j] ** 2).sum()) > B:
            chosen[piv[j]] = True; j += 1; s += 1
        if s == 0: chosen[piv[j]] = True; j += 1
        batches += 1
    return batches
def topm(m):
    def r(dd):
        o = np.argsort(-dd, kind="stable"); return set(o[:m].tolist()), dd[o[m]]
    return r
def perwave(t):
    def r(dd):
        cand = set(); B = -np.inf
        for w in range(8):
            idx = np.nonzero(wave == w)[0]; o = idx[np.argsort(-dd[idx], kind="stable")]
            cand |= set(o[:t].tolist()); B = max(B, dd[o[t]])
        return cand, B
    return r
for CAP in (16, 32, 1000):
    for name, rule in [("wave4", perwave(4)), ("wave8", perwave(8)), ("wave16", perwave(16))]:
        print("cap", CAP, name, run(rule), flush=True)
