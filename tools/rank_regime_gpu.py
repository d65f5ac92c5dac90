"""GPU half of the rank-regime experiment (tests/experiments/rank_rule_c2.py): the C2 build at
c0 = 1e4 (nip = parent rank, every x4_q rank-deficient, the reference demo's regime,
fftisdf.py:455-461) for several fit_tol cuts of the pivoted factorisation; saves the points, the
per-q ranks and J/K per cut to OUT.npz, compared against gelsy on the CPU afterwards
(tests/experiments/rank_rule_c2.py --gpu OUT.npz).

  python tools/rank_regime_gpu.py OUT.npz [TOL ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]
import numpy as np  # noqa: E402


def main(out, tols):
    import bench
    from fisdf import ISDF
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c2")
    res = {}
    for tol in tols:
        df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=1e4)
        df.fit_tol = tol
        d = df.device
        df._kmesh()
        df._ao_parent = d.to_dev(x0)
        df._ao_grid = d.to_dev(chi)
        df.build()
        vj, vk = df.get_jk(dm)
        tag = f"{tol:.1e}"
        res[f"vj_{tag}"], res[f"vk_{tag}"] = vj, vk
        res[f"ranks_{tag}"] = np.asarray(df.ranks)
        res["perm"] = np.asarray(df.perm)
        print(f"fit_tol {tag}: nip {df.nip} ranks {df.ranks.min()}-{df.ranks.max()} "
              f"{df.ranks.tolist()}", flush=True)
    res["tols"] = np.asarray(tols)
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], [float(t) for t in sys.argv[2:]] or [1e-14, 4.2e-15, 3e-15])
