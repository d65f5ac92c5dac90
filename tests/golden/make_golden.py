"""Generate tests/golden/*.npz from the CPU oracle (the reference itself cannot import:
PySCF absent).  Inputs are regenerated deterministically by the tests
from the cell definitions; the fixture holds outputs only.

    python tests/golden/make_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), os.path.dirname(HERE)]

import numpy as np  # noqa: E402

from cases import inputs, oracle  # noqa: E402
from oracle import exact_ref as E, isdf_ref as R  # noqa: E402

for name in ["toy222"]:
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    kpts = R.get_kpts(cell.a, kmesh)
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"), perm=o["perm"], rank=o["rank"], nip=o["nip"],
        ranks=np.asarray(o["ranks"]), vj=o["vj"], vk=o["vk"],
        vj_exact=E.exact_j(chi, dm, cell.a, cell.mesh),
        vk_exact=E.exact_k(chi, dm, cell.a, cell.mesh, kpts, coords),
        w0_diag=np.diag(o["w0"]))
    print(name, "written")
