"""Full-size parity: GPU ISDF build + get_jk vs the CPU oracle (gelsy restatement of
fftisdf.py) on a bench config (default C2; C3 takes a few minutes of CPU).

  python tests/parity_full.py [--config c2|c3|c4|c5] [--no-tr]

Prints one JSON line with max|dJ|, max|dK| (Ha), the ranks and the oracle's CPU time.
The oracle runs with the GPU's interpolation points (SURVEY.md §7 hard part (b))."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--no-tr", action="store_true")
    args = p.parse_args()
    import bench
    from fisdf import ISDF
    from oracle import isdf_ref as R
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup(args.config)
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    df.time_reversal = not args.no_tr
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    t0 = time.perf_counter()
    df.build()
    vj, vk = df.get_jk(dm)
    d.torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    print(f"gpu build+get_jk {tg:.2f} s nip {df.nip} ranks {df.ranks.min()}-{df.ranks.max()}",
          flush=True)
    perm = df.perm
    xip = x0[:, perm]
    coords = cell.gen_uniform_grids(cell.mesh)
    t0 = time.perf_counter()
    out = R.build(xip, chi, coords, cell.a, kmesh, cell.mesh, progress=True)
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    dms = dm[None]
    vj0 = R.get_j_kpts(xip, out["w0"], dms, kpts_band_is_zero=bool(abs(kpts).max() < 1e-9))[0]
    vk0 = R.get_k_kpts(xip, out["wq"], dms, phase)[0]
    tc = time.perf_counter() - t0
    res = dict(config=args.config, time_reversal=not args.no_tr, nip=int(df.nip),
               gpu_ranks=[int(df.ranks.min()), int(df.ranks.max())],
               gelsy_ranks=[int(min(out["ranks"])), int(max(out["ranks"]))],
               dJ=float(abs(vj - vj0).max()), dK=float(abs(vk - vk0).max()),
               maxJ=float(abs(vj0).max()), maxK=float(abs(vk0).max()),
               gpu_s=round(tg, 3), oracle_s=round(tc, 1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
