"""Host-side (Python) time of the C3 bench step: cProfile over K steps of build() + get_jk(),
after W warmup steps — where the step's host hand-offs go (the GPU idles between a step's last
kernel and the next step's first).
  python tools/host_profile.py [--steps 5] [--top 30]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    import torch
    import bench
    from fisdf import ISDF
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c3")
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)

    def step():
        df._dev_state = None
        df.build()
        df.get_jk(dm)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"{(time.perf_counter() - t0) / a.steps * 1e3:.2f} ms/step under cProfile", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(a.top)


if __name__ == "__main__":
    main()
