"""Host hand-offs of the C3 bench step (round 6): the bench's step (build + get_jk) with
FISDF_HOST_TRACE=1 host timestamps from the library and the mirror's own around build() and
get_jk(), on the same clock (CLOCK_MONOTONIC = time.perf_counter).  The device idles from the
moment get_jk's read-back lands (the host returns from get_jk then) until the next build enqueues
its first kernel ("tr check enqueued").
  FISDF_HOST_TRACE=1 python tools/host_gap.py [--steps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
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

    def mark(w):
        print(f"fisdf-host {time.perf_counter():.6f} py: {w}", file=sys.stderr, flush=True)

    for i in range(2 + a.steps):
        mark(f"step {i} start")
        df._dev_state = None
        df.build()
        mark("build() returned")
        df.get_jk(dm)
        mark("get_jk() returned")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
